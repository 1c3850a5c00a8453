set -o pipefail
mkdir -p gpurun_out/prior
timeout -k 10 300 python -u -m pytest tests/test_gpu_pvnet.py -x -q --timeout 240 --timeout-method thread -k "prior" > gpurun_out/prior/t.log 2>&1 || { tail -30 gpurun_out/prior/t.log; exit 1; }
tail -2 gpurun_out/prior/t.log
GZ_AB_CHECK=1 bash tools/r6_ab.sh 2 pbase pnew
