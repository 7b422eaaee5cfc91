# The N-rank bench launch (torchrun, barrier, max-over-ranks, one JSON line)
# rehearsed on a one-GPU box: every rank on cuda:0 over gloo (JH_BENCH_REHEARSE).
#   gpurun -- bash tools/gpu_rehearse_n.sh <outdir> [N]
O=${1:-gpurun_out/rehearse}; N=${2:-2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
JH_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --steps 3 --warmup 1 --no-cpu --e2e 0 > $O/bench_n$N.log 2>&1
