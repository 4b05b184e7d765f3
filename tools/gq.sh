#!/bin/bash
# quick GPU check: parity suite, bench (no cpu legs), stamps
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; tail -3 gpurun_out/$T/pytest.log
timeout -k 10 300 python3 bench.py --cpu-budget 0 --exhaustive-steps 0 --long-run 0 "$@" > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit 1
timeout -k 10 120 python3 tools/stamps.py text:6 text:8 > gpurun_out/$T/stamps.txt 2>&1; cat gpurun_out/$T/stamps.txt
