set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/g1_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/g1_bench_rl.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --family composite_linear > gpurun_out/g1_bench_cl.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --family feature_linear > gpurun_out/g1_bench_fl.log 2>&1
echo "rc=$?"
tail -3 gpurun_out/g1_tests.log; tail -1 gpurun_out/g1_bench_rl.log; tail -1 gpurun_out/g1_bench_cl.log; tail -1 gpurun_out/g1_bench_fl.log
