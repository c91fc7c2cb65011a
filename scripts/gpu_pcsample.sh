# PC-sampling profile of the bench kernel (rocprofv3 beta): where the wave cycles go.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp
M=${1:-stochastic}; U=${2:-cycles}; I=${3:-1048576}
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U --pc-sampling-interval $I -d gpurun_out/pcs -o pcs --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/pcs/bench.json 2> gpurun_out/pcs/bench.err
rc=$?
echo "rc=$rc"; tail -5 gpurun_out/pcs/bench.err; ls -la gpurun_out/pcs
