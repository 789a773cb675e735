#!/bin/bash
# One round's profile set at the BENCH configuration (C2: cover scene, 1920x1080x1024 spp, one frame),
# run on the GPU box from the repo root:
#   1. rocprofv3 kernel trace + stats, two render lanes (the timed bench) and one lane (bench.py's roofline)
#   2. PMC passes over every kernel of one frame (each pass a run of its own, within the per-block limits):
#        fetch: FETCH_SIZE    write: WRITE_SIZE
#        sq1:   VALUBusy VALUUtilization LdsUtil LdsBankConflict OccupancyPercent + SQ_WAIT_ANY SQ_INSTS_LDS
#               SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES (+ GRBM_GUI_ACTIVE)
#        sq2:   SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES + the f64 op counters + SQ_BUSY_CU_CYCLES
#   3. tools/pmc_report.py -> pmc_round.json in the output directory (per kernel family: bytes per item,
#      VALU / LDS busy, lane utilisation, waits), and the extend / shade summaries bench.py reads
#      (profiles/pmc/<scene>_{extend,shade}.json)
# usage: tools/profile_round.sh TAG [extra bench args]
set -e
set -o pipefail
TAG=${1:-r02}
shift || true
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt2 -o kt -- $B > $O/kt2.log 2>&1
echo "kt2 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt1 -o kt -- $B --lanes 1 > $O/kt1.log 2>&1
echo "kt1 ok"
P="$B --no-profile-events"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o f -- $P > $O/fetch.log 2>&1
echo "fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o w -- $P > $O/write.log 2>&1
echo "write ok"
timeout -s KILL 300 rocprofv3 --pmc VALUBusy VALUUtilization LdsUtil LdsBankConflict OccupancyPercent SQ_WAIT_ANY \
  SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/sq1 -o s -- $P > $O/sq1.log 2>&1
echo "sq1 ok"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
  SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/sq2 -o s -- $P > $O/sq2.log 2>&1
echo "sq2 ok"
python3 tools/pmc_report.py $O $O/fetch.log $O/pmc_round.json
cp profiles/pmc/*.json $O/
