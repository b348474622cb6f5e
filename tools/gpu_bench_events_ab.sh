#!/usr/bin/env bash
# bench.py RHS leg A/B: per-step timing events (a copy of the previous bench.py saved as
# tools/bench_prev_events.py for the run, since removed) vs one event pair around the timed steps
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/bench_events_ab.txt
for r in 1 2 3; do for b in 1048576 131072; do for v in bench.py tools/bench_prev_events.py; do
  timeout -k 10 120 python $v --no-cpu-baseline --no-vjp --no-epoch --steps 100 --batch-total $b > gpurun_out/ab_bench.json 2>/dev/null || exit 3
  python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); print('$v', $b, round(d['ms_per_step']*1e3,1), 'us/step wall', round(d['roofline']['kernel_ms']*1e3,1), 'us event', '%.3e' % d['value'])" >> $out
done; done; done
cat $out
