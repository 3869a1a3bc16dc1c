export FKS_NO_AUTOBUILD=1
timeout -k 10 240 python -u tools/gcn_probe.py simple > gpurun_out/gcn_p1.log 2>&1 && \
timeout -k 10 180 python -u tools/gcn_probe.py reference >> gpurun_out/gcn_p1.log 2>&1 && \
timeout -k 10 300 python -u tools/gcn_probe.py children 64 >> gpurun_out/gcn_p1.log 2>&1 && \
timeout -k 10 400 python -u tools/gcn_probe.py bench 64 >> gpurun_out/gcn_p1.log 2>&1
rc=$?; tail -30 gpurun_out/gcn_p1.log; exit $rc
