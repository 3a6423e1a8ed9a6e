# C2 small-batch layer sweep: forced chunk sizes (NONODE_CG) per batch, one bench line each
set -u
cd "${GRAFT_REPO_ROOT}"
O=${O:-gpurun_out/r6c}; mkdir -p $O
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
SPECS=${SPECS:-"8:0 16:0 64:1 64:2 64:3 64:4 128:2 128:4 128:5 256:4 256:5"}
for spec in $SPECS; do
  b=${spec%%:*}; cg=${spec#*:}
  if [ "$cg" = 0 ]; then unset NONODE_CG; else export NONODE_CG=$cg; fi
  timeout -k 10 200 python bench.py --batch $b --steps 30 --no-cpu-baseline > $O/b${b}_cg$cg.json 2>$O/b${b}_cg$cg.err || { echo "bench fail $b $cg"; tail -3 $O/b${b}_cg$cg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b${b}_cg$cg.json')); r=d['roofline']; print('B=$b cg=$cg', round(d['ms_per_step'],4), 'layer', round(r['avg_launch_ms']*1e3,1), 'tconv', round(r['tconv_avg_launch_ms']*1e3,1))"
done
