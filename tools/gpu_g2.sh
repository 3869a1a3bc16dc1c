set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 400 python bench.py --steps 200 --warmup 2 --save-best gpurun_out/best_composite.json > gpurun_out/g2_cl.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 100 --warmup 2 --family feature_linear --save-best gpurun_out/best_feature.json > gpurun_out/g2_fl.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/g2_cl.log; tail -1 gpurun_out/g2_fl.log
