set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/pshade2
mkdir -p $O
python -c "import torch, numpy" || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_shade -f csv -d $O/sfetch -o f -- \
  python3 bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --no-isolated > $O/sfetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_shade -f csv -d $O/swrite -o w -- \
  python3 bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --no-isolated > $O/swrite.log 2>&1 || exit 1
python3 tools/pmc_shade_json.py $O/sfetch/f_counter_collection.csv $O/swrite/w_counter_collection.csv $O/sfetch.log cover profiles/pmc_shade.json || exit 1
cp profiles/pmc_shade.json $O/
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_extend -f csv -d $O/ewrite -o w -- \
  python3 bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --no-isolated > $O/ewrite.log 2>&1 || exit 1
python3 - <<'PY'
import csv, json, os
O=os.environ.get('PWD')+'/gpurun_out/pshade2'
tot=sum(float(r['Counter_Value']) for r in csv.DictReader(open(O+'/ewrite/w_counter_collection.csv')) if r['Counter_Name']=='WRITE_SIZE' and 'k_extend' in r['Kernel_Name'])
d=json.loads([l for l in open(O+'/ewrite.log').read().splitlines() if l.startswith('{')][-1])
print('extend write B/segment', tot*1024/(d['extend_rays_per_step']*d['steps']))
PY
