# 2-rank rehearsal of the bounded self-play on one GPU (gloo), then the single-process check
set -o pipefail
out=gpurun_out/${1:-dist}
mkdir -p $out
GZ_DIST_BACKEND=gloo GZ_DIST_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dist_selfplay_check.py $out > $out/ranks.log 2>&1 &&
timeout -k 10 300 python tools/dist_selfplay_check.py $out > $out/single.log 2>&1
