# BVH variants (continue-with-first-child, 4-wide, per-lane) and the CSG
# search's far-origin shift against the default build; BVH + CSG parity.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_r4_ab.sh ab_csgfar "c4csg" 5 build_variants/librtamd_nocsgfar.so go-raytracer_amd/csrc/librtamd.so || exit 1
bash scripts/gpu_r4_ab.sh ab_bvhv "c5 c4" 5 go-raytracer_amd/csrc/librtamd.so build_variants/librtamd_bvhc.so build_variants/librtamd_bvh4.so build_variants/librtamd_lane.so || exit 1
mkdir -p gpurun_out/r4_par9
timeout -k 10 800 python3 -u -m pytest tests -x -q -m gpu -k "c5 or bvh or c4 or accel or synthetic or csg or extension" --timeout 300 --timeout-method thread > gpurun_out/r4_par9/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4_par9/pytest.log; exit $rc
