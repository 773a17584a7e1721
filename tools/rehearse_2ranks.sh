# Two ranks of bench.py on a one-GPU box (both on cuda:0, gloo collectives):
# the multi-rank path end to end at small sizes.  Not an 8-GPU scaling run.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --no-pmc --keys 2000000 --ensembles 16 --ensemble-keys 200000 \
  --part-keys 20000000 --part-batches 4 --part-batch-keys 200000 > gpurun_out/r06_2ranks.json 2> gpurun_out/r06_2ranks.err
rc=$?; tail -5 gpurun_out/r06_2ranks.err; head -c 600 gpurun_out/r06_2ranks.json; exit $rc
