#!/bin/bash
# Attribution of the durable headline: cProfile of the default run, then variants that drop one
# stage each.  Results under gpurun_out/<name>.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_attrib}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
S=40
timeout -k 10 300 python -u -m cProfile -o "$O/prof.out" bench.py --steps $S --warmup 5 > "$O/default.log" 2>&1 || exit 1
python -c "import pstats; p=pstats.Stats('$O/prof.out'); p.sort_stats('tottime').print_stats(25)" > "$O/prof_tottime.txt" 2>&1
python -c "import pstats; p=pstats.Stats('$O/prof.out'); p.sort_stats('cumulative').print_stats(40)" > "$O/prof_cum.txt" 2>&1
for v in "--no-durable" "--no-alt-ids" "--p-unregistered 0 --p-register 0 --p-ack 0" "--no-alt-ids --p-unregistered 0 --p-register 0 --p-ack 0 --no-durable"; do
  n=$(echo "$v" | tr -d ' -' | cut -c1-40)
  timeout -k 10 300 python -u bench.py --steps $S --warmup 5 $v > "$O/v_$n.log" 2>&1 || exit 1
  echo "$v: $(tail -1 "$O/v_$n.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "M/s", d["ms_per_step"], "ms")')"
done
tail -1 "$O/default.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("default:", round(d["value"]/1e6,1), "M/s", d["ms_per_step"], "ms")'
