# Round 6: the multi-device Render() seam (rt_render_ex), compile-free first
# calls, the hipRTC environment regression, the C host.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_seam}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_render_ex.py tests/test_gpu_render_api.py tests/test_c_host.py -x -v -s -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "first call|passed|failed" $O/pytest.log | tail -8
