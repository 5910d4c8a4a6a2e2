# default bench (N=1) + an N=2 rehearsal of the sharded path on the one GPU (gloo)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r03d_bench.json; tail -3 gpurun_out/r03d_bench.err; [ $rc -eq 0 ] || exit $rc
SB_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --no-cpu --no-encode --no-b12 --no-hard --rows 20000000 --c3-rows 10000000 --c4-rows 5000000 --c5-rows 1048576 > gpurun_out/r03d_n2.json 2> gpurun_out/r03d_n2.err
rc=$?; echo "n2 rc=$rc"; tail -c 1200 gpurun_out/r03d_n2.json; tail -5 gpurun_out/r03d_n2.err; exit $rc
