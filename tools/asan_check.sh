#!/bin/bash
# Host-sanitized CPU check: the C / C++ host code
# (IntVector twin, sharded driver argument paths, apps, oracle) built with gcc
# ASan + UBSan (make asan, oracle liboracle_asan.so), then the CPU tests that
# exercise it run against those builds with gcc's runtimes preloaded into
# Python.  Any ASan / UBSan report fails the run (halt_on_error, and UBSan
# built with -fno-sanitize-recover).  Leak checking is off: CPython and torch
# keep their allocations until exit.
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C mpi-k-selection_amd asan
make -s -C oracle liboracle_asan.so
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
export LD_PRELOAD="$(readlink -f "$ASAN_RT"):$(readlink -f "$UBSAN_RT")"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export KTH_LIB=$PWD/mpi-k-selection_amd/lib/asan/libkth.so
export KTH_ORACLE_LIB=$PWD/oracle/liboracle_asan.so
export KTH_BIN_DIR=$PWD/mpi-k-selection_amd/bin/asan
python -m pytest -x -q -m "not gpu" -p no:cacheprovider \
    tests/test_abi.py tests/test_oracle_golden.py tests/test_seq_driver.py tests/test_cgm_driver.py "$@"
