#!/bin/bash
# SQ counters of k_extend per closest-hit mode (flat list / wave-uniform BVH /
# per-lane BVH).  Run on the GPU box from the repo root.
export TMPDIR=/tmp
R=$PWD
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY"
for mode in flat wave lane; do
  if [ $mode = flat ]; then export RTAMD_BVH_MIN=1000000000; else export RTAMD_BVH_MIN=1; export RTAMD_TRAVERSAL=$mode; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex k_extend -f csv -d $R/gpurun_out/pmc_$mode$i -o p -- \
      python3 bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events > gpurun_out/pmc_$mode$i.log 2>&1 || exit $?
  done
done
