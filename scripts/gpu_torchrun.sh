# Driver-style launch of the bench at N=1 (torchrun, RCCL process group, two frames in flight),
# plus the weak-scaling path and a serial (--inflight 1) line for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/torchrun}
mkdir -p $O
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 30 --warmup 3 --cpu-baseline off > $O/torchrun_n1.json 2> $O/torchrun_n1.err || { tail -5 $O/torchrun_n1.err; exit 1; }
cat $O/torchrun_n1.json
timeout -k 10 300 python3 bench.py --scaling weak --cpu-baseline off --companion off > $O/weak_n1.json 2> $O/weak_n1.err || { tail -5 $O/weak_n1.err; exit 1; }
timeout -k 10 300 python3 bench.py --inflight 1 --cpu-baseline off --companion off > $O/serial_n1.json 2> $O/serial_n1.err || { tail -5 $O/serial_n1.err; exit 1; }
python3 -c "
import json
for f in ('torchrun_n1','weak_n1','serial_n1'):
    d=json.load(open('$O/%s.json'%f)); print(f, d['ms_per_step'], d['value'], d['config']['parallelism'], d['config']['frames_in_flight'], d['roofline']['kernel_ms'])"
