#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each, <= 8 SQ counters) over a bench workload (WL, default egno = C2), then a per-kernel
# summary (tools/pmc_summary.py). NONODE_LIB passes through.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/prof_${TAG:-pmc}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload ${WL:-egno} --steps 5 --warmup 1 --no-cpu-baseline --no-kernel-events > /dev/null 2>$OUT/trace.err || exit $?
i=0
for pass in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY" \
            "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MISC" \
            "SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $OUT/pmc_p$i -o run -- python3 bench.py --workload ${WL:-egno} --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-events > /dev/null 2>$OUT/pmc_p$i.err
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/pmc_p$i.err; exit $rc; }
done
python3 tools/pmc_summary.py $OUT -v
