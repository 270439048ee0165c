# Round-end check: the whole -m gpu suite, smoke, the default bench line, and the
# 2-rank gloo rehearsal of the sharded path on one GPU (reassembly checked).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-final}
bash tools/gpu_session.sh $TAG || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --check 3000 --no-cpu --no-extra \
  > gpurun_out/rehearsal_2_$TAG.json 2> gpurun_out/rehearsal_2_$TAG.err || exit 1
