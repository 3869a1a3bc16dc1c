#!/bin/bash
# Parameterised GPU session driver (run through gpurun on the MI355X box):
#
#   tools/gpu_check.sh NAME STEP [STEP ...]
#
# Every step runs under its own time limit; the first failure ends the call
# (nothing more touches the GPU after a fault, abort or timeout).  Output goes
# to gpurun_out/NAME/.  Steps:
#
#   tests[=ARGS]        pytest -m gpu (ARGS: test files / -k expression instead of the whole suite)
#   smoke               __graft_entry__.smoke()
#   bench[=ARGS]        python bench.py ARGS            -> bench.json
#   prof[=ARGS]         rocprofv3 --kernel-trace --stats of bench.py ARGS -> prof/
#   steady=SECS[:CFG[:GENS]]  steady-state program islands for SECS seconds (CFG: configs/config3_steady.json;
#                       GENS: generation target, so a long run keeps producing children)
#   rccl[=ARGS]         tools/rccl_check.py (default --steady-s 0: no producer processes under the profiler)
#                       under rocprofv3 --kernel-trace --stats -> rccl.log, rccl_prof/
#   native=ARGS         tools/native_bench.py ARGS      -> native.jsonl
#   c5[=ARGS]           config-5 bench (synthetic 65,536 pods / 256 nodes) -> c5.json
#   pmc=COUNTERS[:ARGS] one rocprofv3 --pmc pass over bench.py ARGS (counters comma-separated)
#   py=SCRIPT[:ARGS]    python SCRIPT ARGS              -> py_<script>.txt  (ARGS comma-separated)
#   avail               rocprofv3 --list-avail          -> avail.txt
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
NAME=$1
shift
O=gpurun_out/$NAME
mkdir -p "$O"

die() { echo "FAILED: $1"; [ -f "$2" ] && tail -40 "$2"; exit 1; }

for step in "$@"; do
  key=${step%%=*}
  val=""
  [ "$key" != "$step" ] && val=${step#*=}
  echo "== $step ($(date +%T))"
  case $key in
    tests)
      [ -z "$val" ] && val=tests
      timeout -k 10 900 python -u -m pytest ${val//,/ } -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$O/gpu_tests.txt" 2>&1 || die tests "$O/gpu_tests.txt"
      tail -2 "$O/gpu_tests.txt" ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 \
        || die smoke "$O/smoke.txt"
      tail -1 "$O/smoke.txt" ;;
    bench)
      timeout -k 10 600 python -u bench.py ${val//,/ } > "$O/bench.json" 2> "$O/bench.err" || die bench "$O/bench.err"
      cut -c1-400 "$O/bench.json" ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py ${val:---steps 3 --warmup 1 --programs 0 --novel 0 --novel-large 0 --evolved 0} \
        > "$O/prof.log" 2>&1 || die prof "$O/prof.log"
      echo "profile written" ;;
    steady)
      secs=${val%%:*}
      cfg=configs/config3_steady.json
      gens=""
      if [ "$secs" != "$val" ]; then
        rest=${val#*:}
        cfg=${rest%%:*}
        [ "$cfg" != "$rest" ] && gens="--generations ${rest#*:}"
        [ -z "$cfg" ] && cfg=configs/config3_steady.json
      fi
      timeout -k 10 $((secs + 240)) python -u -m funsearch_kubernetes_simulator_amd.funsearch --config "$cfg" $gens \
        --verbose --wall-s "$secs" --save "$O/top5.json" --checkpoint-dir "$O/ck" --metrics-log "$O/metrics.jsonl" \
        > "$O/steady.log" 2>&1 || die steady "$O/steady.log"
      grep steady_final "$O/steady.log" | cut -c1-600 ;;
    rccl)
      # one-rank RCCL group beside the replay slots, under a kernel trace (RCCL kernels next to the replay kernel)
      FKS_DIST_GROUP=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29731 \
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/rccl_prof" -o run -- python3 tools/rccl_check.py \
        ${val:---steady-s 0} > "$O/rccl.log" 2>&1 || die rccl "$O/rccl.log"
      grep '^{' "$O/rccl.log" | tail -1 | cut -c1-400 ;;
    native)
      timeout -k 10 400 python -u tools/native_bench.py $val > "$O/native.jsonl" 2>&1 || die native "$O/native.jsonl"
      tail -3 "$O/native.jsonl" | cut -c1-300 ;;
    c5)
      timeout -k 10 600 python -u bench.py --trace synthetic --programs 0 --novel 0 --novel-large 0 --evolved 0 ${val:---steps 3 --warmup 1 --candidates 4096} \
        > "$O/c5.json" 2> "$O/c5.err" || die c5 "$O/c5.err"
      cut -c1-300 "$O/c5.json" ;;
    pmc)
      ctrs=${val%%:*}
      args="--steps 2 --warmup 1 --programs 0 --novel 0 --novel-large 0 --evolved 0"
      [ "$ctrs" != "$val" ] && args=${val#*:}
      timeout -s KILL 120 rocprofv3 --pmc ${ctrs//,/ } -d "$O/pmc_${ctrs//,/_}" -o run -- python3 bench.py $args \
        > "$O/pmc_${ctrs//,/_}.log" 2>&1 || die pmc "$O/pmc_${ctrs//,/_}.log"
      echo "pmc pass written" ;;
    py)
      script=${val%%:*}
      args=""
      [ "$script" != "$val" ] && args=${val#*:}
      args=${args//,/ }   # (commas separate the script's arguments)
      base=$(basename "$script" .py)
      out="$O/py_$base.txt"
      n=2
      while [ -e "$out" ]; do out="$O/py_${base}_$n.txt"; n=$((n + 1)); done   # repeated steps keep their output
      timeout -k 10 900 python -u "$script" $args > "$out" 2>&1 || die "py $script" "$out"
      tail -5 "$out" | cut -c1-400 ;;
    avail)
      # the PMC counters this rocprofv3 / gfx950 exposes (names for pmc= passes)
      timeout -s KILL 60 rocprofv3 --list-avail > "$O/avail.txt" 2>&1 || die avail "$O/avail.txt"
      grep -c . "$O/avail.txt" ;;
    *)
      die "unknown step $step" ;;
  esac
done
echo "== done ($(date +%T))"
