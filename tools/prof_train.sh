set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train/trace -o run -- python3 bench.py --workload egno_train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_train/bench.json 2> gpurun_out/prof_train/err.txt
echo rc=$?
