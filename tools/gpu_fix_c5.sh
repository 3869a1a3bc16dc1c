# Validate the JIT-compiler race fix (native GPU tests + a resumed config-3 run), then a config-5 heap-top sweep.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fix gpurun_out/c5
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/fix/tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fix/tests.txt; exit 1; }
tail -4 gpurun_out/fix/tests.txt
cp runs/config3_native/islands_rank0.json runs/config3_native/metrics.jsonl gpurun_out/fix/
timeout -k 10 200 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_native.json \
  --generations 10 --resume --checkpoint-dir gpurun_out/fix --log gpurun_out/fix/metrics.jsonl \
  --save gpurun_out/fix/top5.json > gpurun_out/fix/run.log 2>&1 || { echo "resume failed"; tail -20 gpurun_out/fix/run.log; exit 1; }
tail -1 gpurun_out/fix/run.log | cut -c1-300
for ht in ${HTS:-1023 511 255 127}; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates 1536 --steps 2 --warmup 1 --programs 0 --heap-top $ht \
    > gpurun_out/c5/ht_$ht.json 2> gpurun_out/c5/ht_$ht.err || { echo "bench ht=$ht failed"; tail -20 gpurun_out/c5/ht_$ht.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c5/ht_$ht.json')); print('heap_top', $ht, d['value'], d['ms_per_step'])"
done
# PMC counters of one config-5 launch (own pass per counter group; each pass under a hard time limit)
mkdir -p gpurun_out/pmc5
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --kernel-trace -d gpurun_out/pmc5/a -o run --output-format csv -- python3 tools/pmc_c5_driver.py 2048 \
  > gpurun_out/pmc5/a.log 2>&1 || { echo "pmc pass a failed"; tail -5 gpurun_out/pmc5/a.log; exit 1; }
tail -1 gpurun_out/pmc5/a.log | cut -c1-200
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
  --kernel-trace -d gpurun_out/pmc5/b -o run --output-format csv -- python3 tools/pmc_c5_driver.py 2048 \
  > gpurun_out/pmc5/b.log 2>&1 || { echo "pmc pass b failed"; tail -5 gpurun_out/pmc5/b.log; exit 1; }
echo pmc done
