# Throughput/size sweep over parse settings (diagnostic; each line = one bench run).
# SWEEP="K:lazy ..." overrides the list; NOWL=1 skips the zeros/random lines.
B="timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-budget 0 --exhaustive-steps 0"
show='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ratio"], d["stage_ms"])'
for cfg in ${SWEEP:-1:0 4:0 8:0 16:0 0:0 4:1 6:1 8:1 16:1 0:1}; do
  k=${cfg%:*}; lz=${cfg#*:}
  $B --max-chain $k --lazy $lz 2>/dev/null | python3 -c "$show" "text mc=$k lazy=$lz"
done
[ -n "${NOWL:-}" ] || for w in zeros random; do $B --workload $w 2>/dev/null | python3 -c "$show" "$w"; done
