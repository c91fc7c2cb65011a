set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RT_AMD_LIB=build_variants/librtamd_cost.so timeout -k 10 300 python scripts/cost_map.py c5 480 270 gpurun_out/cost_c5.npy > gpurun_out/cost_c5.log 2>&1
