set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r6b; mkdir -p $O
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_parity.py tests/test_gpu_options.py tests/test_gpu_train_segno.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?"; grep -E "^FAILED|^ERROR|passed|failed" $O/pytest_gpu.log | tail -8
for rep in 1 2; do
for b in 64 128 256; do
  for mode in crit fill; do
    if [ $mode = fill ]; then export NONODE_FILL_CG=1; else unset NONODE_FILL_CG; fi
    timeout -k 10 200 python bench.py --batch $b --steps 50 --no-cpu-baseline > $O/b${b}_${mode}_$rep.json 2>$O/b${b}_${mode}.err || { echo "bench fail $b $mode"; tail -3 $O/b${b}_${mode}.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b${b}_${mode}_$rep.json')); r=d['roofline']; h=d['host_overhead']; print('$b $mode', round(d['ms_per_step'],4), round(r['avg_launch_ms']*1e3,1), 'host', round(h['enqueue_ms_median'],3), round(h['sync_wall_ms_median'],3), round(h['recorded_kernel_ms_per_call'],3))"
  done
done
done
unset NONODE_FILL_CG
