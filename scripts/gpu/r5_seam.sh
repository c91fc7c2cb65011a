# Round 5: rt_render seam tests + band/thread sweep + default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_seam}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_render_api.py \
  "tests/test_gpu_parity.py::test_csg_leaf_groups_and_far_origins_match_oracle" \
  "tests/test_gpu_parity.py::test_rt_render_repeated_calls_equal_oracle" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python3 scripts/api_seam.py > $O/api_seam.log 2>&1 || { tail -5 $O/api_seam.log; exit 1; }
cat $O/api_seam.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
