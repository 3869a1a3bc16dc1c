#!/bin/bash
# Equal-wall-time A/B of the MFMA surrogate pre-filter: for each seed,
# the default bench config with --screen 1 (exact replay only) and --screen 4 (4x proposals,
# MFMA-screened to the best 1/4, surrogate states re-drawn from the elites every epoch).
# Result lines -> gpurun_out/screen_ab/ab.jsonl; summary: python tools/screen_ab_summary.py
set -o pipefail
export FKS_NO_AUTOBUILD=1
BUDGET=${BUDGET:-45}
mkdir -p gpurun_out/screen_ab
out=gpurun_out/screen_ab/ab.jsonl
: > $out
for seed in 11 22 33 44 55; do
  for k in 1 4; do
    timeout -k 10 240 python -u bench.py --time-budget $BUDGET --warmup 1 --screen $k --seed $seed \
      --programs 0 --novel 0 > gpurun_out/screen_ab/s${seed}_k${k}.json 2> gpurun_out/screen_ab/s${seed}_k${k}.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'seed': int(sys.argv[2]), 'k': int(sys.argv[3]), 'best_score': d['best_score'], 'value': d['value'], 'steps': d['steps'], 'screen': d.get('screen')}))" gpurun_out/screen_ab/s${seed}_k${k}.json $seed $k >> $out
    tail -1 $out | cut -c1-200
  done
done
