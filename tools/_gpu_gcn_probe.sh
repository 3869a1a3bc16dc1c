# staged MI355X check of the baseline JIT (each stage bounded; stop at the first failure)
export FKS_NO_AUTOBUILD=1
out=gpurun_out/gcn_probe.log
timeout -k 10 240 python -u tools/gcn_probe.py simple > $out 2>&1 && \
timeout -k 10 180 python -u tools/gcn_probe.py reference >> $out 2>&1 && \
timeout -k 10 300 python -u tools/gcn_probe.py children 96 >> $out 2>&1 && \
timeout -k 10 400 python -u tools/gcn_probe.py bench 64 >> $out 2>&1 && \
timeout -k 10 400 python -u tools/gcn_probe.py bench 256 >> $out 2>&1
rc=$?; grep -v amdgpu.ids $out | tail -30; exit $rc
