set -o pipefail
mkdir -p gpurun_out
RTAMD_DEBUG_COUNTS=1 RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_stats.so timeout -k 10 200 python tools/trav_stats.py cover 2 > gpurun_out/trav_stats.json 2> gpurun_out/trav_stats.err || { tail gpurun_out/trav_stats.err; exit 1; }
cat gpurun_out/trav_stats.json | grep -v "^  *\"\(lane\|wave\|lanes\)"
grep "neighbours" gpurun_out/trav_stats.err | sort | uniq -c | head
