# the sharded protocol at world 1 (RCCL): per-select time and its kernel timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 180 python -u bench.py --dist --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/dist1.log 2>&1 || { echo rc=$?; tail -20 gpurun_out/dist1.log; exit 1; }
tail -1 gpurun_out/dist1.log | cut -c1-400
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof -o run --output-format csv -- python3 bench.py --dist --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dprof.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/dprof.log; exit 1; }
python3 - <<'PY'
import csv
rows = sorted(csv.DictReader(open('gpurun_out/dprof/run_kernel_trace.csv')), key=lambda r: int(r['Start_Timestamp']))
ks = [r for r in rows if 'k_gather' in r['Kernel_Name'] or 'kth::' in r['Kernel_Name'] or 'nccl' in r['Kernel_Name'].lower()]
starts = [i for i, r in enumerate(ks) if 'k_gather' in r['Kernel_Name']]
seq = ks[starts[-2]:starts[-1]]
t0 = int(seq[0]['Start_Timestamp'])
for r in seq:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"  {r['Kernel_Name'].split('(')[0][:40]:40s} {(e - s) / 1000:8.1f} us  +{(s - t0) / 1000:8.1f} -> +{(e - t0) / 1000:8.1f}")
PY
