# Round 4 (k): the row loop's grid (workgroups per CU) against the one-row-per-wave build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4k; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
L=mpi-k-selection_amd/lib
python3 - <<'PY'
import ctypes, torch
import sys; sys.path.insert(0, "mpi-k-selection_amd")
PY
run() {  # label env...
  lab=$1; shift
  for args in "--rows-dtype i32" "--rows-dtype i32 --topk"; do
    env "$@" timeout -k 10 120 python -u bench.py --workload rows $args --k 64 --steps 20 --warmup 3 --no-cpu-baseline > $O/rows.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/rows.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/rows.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$lab', '$args', round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us', d['verified'])"
  done
}
run noloop KTH_LIB=$L/variants/libkth_noloop.so
for pc in 1 2 3 4 5 6 8 16; do run "loop pc=$pc" KTH_ROWS_GRID_PER_CU=$pc; done
run "loop auto" KTH_ROWS_GRID_PER_CU=0
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload rows --rows-dtype i32 --k 64 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof rc=$?; tail -5 $O/prof.log; exit 1; }
python3 - <<'PY'
import csv
rows = [r for r in csv.DictReader(open("gpurun_out/r4k/prof/run_kernel_trace.csv")) if "k_rows_reg" in r["Kernel_Name"]]
r = rows[-1]
print({k: r[k] for k in r if k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size", "Arch_VGPR_Count")})
PY
echo done
