# kernel-trace A/B of two libmpcx builds on config-2 launches (timing-only variants)
set -o pipefail
mkdir -p gpurun_out/ab_time && export TMPDIR=/tmp
for i in 1 2; do
  for l in base nomul; do
    f=mpcium_amd/libmpcx.so; [ $l = nomul ] && f=build/ab/libmpcx_nomul.so
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_time/$l$i -o t -- python3 tools/ab_time.py $f 6 > /dev/null 2>&1 || exit 1
    python3 -c "
import csv,glob
f=glob.glob('gpurun_out/ab_time/$l$i/**/t_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'k_modexp<4, 37' in r['Name']: print('$l', $i, r['Calls'], round(float(r['AverageNs'])/1e6, 3), round(float(r['MinNs'])/1e6, 3))"
  done
done
