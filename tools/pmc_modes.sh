#!/bin/bash
# SQ counters of k_extend for one scene (run on the GPU box from the repo root).
# usage: tools/pmc_modes.sh SCENE SPP [flat]   (flat: brute-force list, no BVH)
export TMPDIR=/tmp
R=$PWD
SCENE=${1:-cover}
SPP=${2:-8}
MODE=${3:-bvh}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY"
P3="SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_WAIT_INST_LDS"
P4="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum"
P5="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
P6="SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_LEVEL_LDS"
if [ "$MODE" = flat ]; then export RTAMD_BVH_MIN=1000000000; else export RTAMD_BVH_MIN=1; fi
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5" "$P6"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex ${KREGEX:-k_extend} -f csv -d $R/gpurun_out/pmc_${SCENE}_$MODE$i -o p -- \
    python3 bench.py --scene $SCENE --spp $SPP --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events \
    > gpurun_out/pmc_${SCENE}_$MODE$i.log 2>&1 || exit $?
done
