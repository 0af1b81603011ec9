# two-rank rehearsal of the N > 1 bench path on the one-GPU box (ranks share the device, gloo timing)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-e2e --no-configs --no-ab > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { echo N2_FAIL; tail -30 gpurun_out/bench_n2.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_n2.json').read().strip().splitlines()[-1]); print(d['n_gpus'], round(d['value']/1e6,1), d['ms_per_step'], d['config'])"
