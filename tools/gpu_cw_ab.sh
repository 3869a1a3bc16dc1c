# A/B: program bytecode compiles in-process vs in 8 spawned workers (device.compile_workers), fresh
# coupled config-3 runs of G generations each (two-wave native kernel in both).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cw
G=${G:-300}
for cw in 0 8; do
  python - "$cw" <<'PY'
import json, sys
c = json.load(open("configs/config3_coupled.json"))
c["device"]["compile_workers"] = int(sys.argv[1])
c["checkpoint"] = {"dir": f"gpurun_out/cw/ck{sys.argv[1]}", "every": 100}
c["log_path"] = f"gpurun_out/cw/metrics_cw{sys.argv[1]}.jsonl"
json.dump(c, open(f"gpurun_out/cw/cfg{sys.argv[1]}.json", "w"))
PY
  timeout -k 10 400 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config gpurun_out/cw/cfg$cw.json \
    --generations $G --verbose > gpurun_out/cw/run_cw$cw.log 2>&1 || { echo "run cw=$cw failed"; tail -20 gpurun_out/cw/run_cw$cw.log; exit 1; }
  echo "cw=$cw"; grep '"kind": "generation"' gpurun_out/cw/metrics_cw$cw.jsonl | tail -1 | cut -c1-420
done
