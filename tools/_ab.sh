set -o pipefail
O=gpurun_out/ab1; mkdir -p $O
timeout -k 10 300 python -u tools/ab_env.py --spp 256 --rounds 3 --lanes 1 base: no_solo:RTAMD_NO_SOLO=1 > $O/l1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_env.py --spp 256 --rounds 3 --lanes 2 base: no_solo:RTAMD_NO_SOLO=1 > $O/l2.log 2>&1 || exit 1
cat $O/l1.log $O/l2.log | grep variant
