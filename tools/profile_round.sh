#!/bin/bash
# One round's profile set (run on the GPU box from the repo root):
#  1. rocprofv3 kernel trace + stats of bench.py at 256 spp, and single-lane at the default 1024 spp
#  2. PMC FETCH_SIZE, WRITE_SIZE and SQ f64 passes over k_extend (8 spp)
#  3. profiles/pmc_extend.json from 2.
#  4. PMC FETCH_SIZE, WRITE_SIZE over k_shade (8 spp) -> profiles/pmc_shade.json
# usage: tools/profile_round.sh TAG
set -e
TAG=${1:-r01}
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- \
  python3 bench.py --spp 256 --steps 1 --warmup 0 --no-cpu-baseline --no-isolated > $O/kt.log 2>&1
# the bench's own configuration (1024 spp) with one render lane: its per-launch
# kernel durations are what roofline_isolated measures with HIP events
RTAMD_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_l1_full -o kt -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated > $O/kt_l1_full.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_extend -f csv -d $O/fetch -o f -- \
  python3 bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --no-isolated > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_extend -f csv -d $O/write -o w -- \
  python3 bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --no-isolated > $O/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU \
  --kernel-include-regex k_extend -f csv -d $O/sq -o s -- \
  python3 bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --no-isolated > $O/sq.log 2>&1
python3 tools/pmc_to_json.py $O/fetch/f_counter_collection.csv $O/write/w_counter_collection.csv $O/fetch.log cover \
  profiles/pmc_extend.json $O/sq/s_counter_collection.csv
cp profiles/pmc_extend.json $O/
# 4. the same two byte counters over the shade kernels -> profiles/pmc_shade.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_shade -f csv -d $O/sfetch -o f -- \
  python3 bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --no-isolated > $O/sfetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_shade -f csv -d $O/swrite -o w -- \
  python3 bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --no-isolated > $O/swrite.log 2>&1
python3 tools/pmc_shade_json.py $O/sfetch/f_counter_collection.csv $O/swrite/w_counter_collection.csv $O/sfetch.log cover \
  profiles/pmc_shade.json
cp profiles/pmc_shade.json $O/
