#!/bin/bash
# One GPU-box probe (diagnostic): a -m gpu subset, then optional steps, each under its own
# time limit; the first failure (other than failed tests) ends the script.
# usage (on the box): bash tools/gq.sh TAG PYTEST_K [step ...]
#   steps: bench[:ARGS]  st:[libv=NAME,]MB,K,FLAGS,KIND  ktrace:MB,K,FLAGS,KIND  stamps[:CFGS]  sq[:ARGS]  inflate[:ARGS]  infpmc[:ARGS]  deep  trace[:ARGS]
set -uo pipefail
TAG=$1; K=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$K" != "-" ]; then
  timeout -k 10 600 python3 -u -m pytest "$R/tests" -m gpu -x -q -p no:cacheprovider --timeout 240 \
      --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "pytest status $rc: stopping"; exit $rc; fi
fi
nb=0
for st in "$@"; do
  name=${st%%:*}; arg=""; [ "$name" != "$st" ] && arg=${st#*:}
  case $name in
    bench) nb=$((nb + 1)); bj=$OUT/bench$([ $nb -gt 1 ] && echo $nb).json
           timeout -k 10 600 python3 "$R/bench.py" ${arg//,/ } > "$bj" 2> "${bj%.json}.err" || exit 3
           python3 - "$bj" <<'PY'
import json, sys; d = json.load(open(sys.argv[1]))
print('value', d['value'], 'size', d.get('size_vs_ref_pct'), 'parity', d.get('parity_vs_port'), 'stage', d['stage_ms'])
for k in ('exhaustive', 'real_text', 'gpu_inflate', 'end_to_end_fd_api'):
    v = d.get(k); print(k, {x: v.get(x) for x in ('value', 'GBps_out', 'size_vs_ref_pct', 'parity_vs_port', 'bit_exact')} if v else None)
print('tradeoff', [(t['max_chain'], t['value'], t.get('size_vs_ref_pct')) for t in (d.get('tradeoff') or [])])
PY
           ;;
    stamps) timeout -k 10 300 python3 "$R/tools/stamps.py" ${arg//,/ } > "$OUT/stamps.txt" 2>&1 || exit 3; cat "$OUT/stamps.txt" ;;
    sq) bash "$R/tools/sq_profile.sh" "$TAG/sq" ${arg//,/ } > /dev/null 2>&1 || exit 3; cat "$OUT/sq/sq_summary.txt" ;;
    inflate) timeout -k 10 300 python3 "$R/tools/inflate_bench.py" ${arg//,/ } > "$OUT/inflate.json" 2>&1 || exit 3; cat "$OUT/inflate.json" ;;
    infpmc) cd /tmp; for set in "FETCH_SIZE" "WRITE_SIZE"; do
              timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/ipmc_$set" -o p -- python3 "$R/tools/inflate_bench.py" --steps 2 --stream-mb 1 ${arg//,/ } > /dev/null 2> "$OUT/ipmc_$set.err" || exit 3
            done; python3 "$R/tools/pmc.py" "$OUT/ipmc_FETCH_SIZE,$OUT/ipmc_WRITE_SIZE" | tee "$OUT/inf_pmc.txt"; cd "$R" ;;
    st) a2=${arg//,/ }; lv=""   # stage_time.py [libv=NAME] MB K FLAGS KIND
        if [[ $a2 == libv=* ]]; then lv=${a2%% *}; lv=${lv#libv=}; a2=${a2#* }; fi
        ( [ -n "$lv" ] && export DMX_LIBV="$R/build/var/libdmx_$lv.so"; timeout -k 10 300 python3 "$R/tools/stage_time.py" $a2 ) >> "$OUT/stage_time.txt" 2>&1 || exit 3
        tail -1 "$OUT/stage_time.txt" ;;
    ktrace) cd /tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktrace_$nb" -o run -- python3 "$R/tools/stage_time.py" ${arg//,/ } >> "$OUT/ktrace.txt" 2>&1 || exit 3
           f=$(find "$OUT/ktrace_$nb" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_$nb.csv"; cut -d, -f1-4 "$OUT/kernel_stats_$nb.csv" | head -14; nb=$((nb + 1)); cd "$R" ;;
    pipe) a2=${arg//,/ }; lv=""   # pipe_time.py [libv=NAME] MB K FLAGS KIND STEPS
        if [[ $a2 == libv=* ]]; then lv=${a2%% *}; lv=${lv#libv=}; a2=${a2#* }; fi
        ( [ -n "$lv" ] && export DMX_LIBV="$R/build/var/libdmx_$lv.so"; timeout -k 10 300 python3 "$R/tools/pipe_time.py" $a2 ) >> "$OUT/pipe.txt" 2>&1 || exit 3
        tail -1 "$OUT/pipe.txt" ;;
    fdchunk) a2=${arg//,/ }; lv=""   # fd_chunk.py [libv=NAME] MB CHUNK_MB ...
        if [[ $a2 == libv=* ]]; then lv=${a2%% *}; lv=${lv#libv=}; a2=${a2#* }; fi
        ( [ -n "$lv" ] && export DMX_LIBV="$R/build/var/libdmx_$lv.so"; timeout -k 10 300 python3 "$R/tools/fd_chunk.py" $a2 ) >> "$OUT/fdchunk.txt" 2>&1 || exit 3
        grep chunk_mb "$OUT/fdchunk.txt" | tail -3 ;;
    deep) lv=${arg#libv=}   # deep[:libv=NAME]
        ( [ -n "$arg" ] && export DMX_LIBV="$R/build/var/libdmx_$lv.so"; timeout -k 10 300 python3 "$R/tools/deep_bench.py" 32 ) >> "$OUT/deep.txt" 2>&1 || exit 3
        grep -v amdgpu "$OUT/deep.txt" | tail -4 ;;
    trace) cd /tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-budget 0 --exhaustive-steps 0 --tradeoff= --long-run 0 ${arg//,/ } > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit 3
           find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; ; cut -d, -f1-8 "$OUT/kernel_stats.csv" | head -20; cd "$R" ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
