set -o pipefail
mkdir -p gpurun_out/evf
bash profiles/collect.sh r03c &&
bash tools/clock_probe.sh gpurun_out/evf/clk tree $PWD/alphazero-gomoku_amd/gzero/libgzero.so &&
GZ_DIST_SAME_DEVICE=1 GZ_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --slots 1024 --steps 6 --warmup 2 --burn-in 200 > gpurun_out/evf/dist2.json 2> gpurun_out/evf/dist2.err
