# Packed FP32 child-box tests (RT_BVH_PK, interleaved nodes) vs the unpacked
# build; BVH parity with the packed default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_r4_ab.sh ab_pk "c5 c4" 5 build_variants/librtamd_nopk.so go-raytracer_amd/csrc/librtamd.so || exit 1
mkdir -p gpurun_out/r4_pkpar
timeout -k 10 800 python3 -u -m pytest tests -x -q -m gpu -k "c5 or bvh or c4 or accel or synthetic" --timeout 300 --timeout-method thread > gpurun_out/r4_pkpar/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4_pkpar/pytest.log; exit $rc
