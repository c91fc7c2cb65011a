# Round 5: brute-force C5 (config 5 as stated: no BVH, no culling) --
# uniform-scale sphere runs; parity, the full-width strips and the full 8K
# frame, then the row band 2048-2304 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_brute}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_synthetic_goldens.py \
  tests/test_gpu_parity.py -k "brute or axis or synthetic or full_size_strip or full_frame" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python3 bench.py --config c5 --accel none --rows 2048:2304 --steps 2 --warmup 1 --cpu-baseline off > $O/band.json 2> $O/band.err || { tail -5 $O/band.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/band.json')); r=d['roofline']
print('band ms/step', d['ms_per_step'], 'ref-work frac', r.get('reference_work_frac'), 'achieved TF', r.get('achieved'))"
