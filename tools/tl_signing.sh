set -o pipefail
O=gpurun_out/r05/tl1; mkdir -p $O
for lib in build/hv_r5base/libmpcx_host.so mpcium_amd/libmpcx_host.so; do
  tag=$(basename $(dirname $lib))
  cp mpcium_amd/libmpcx_host.so $O/orig.so
  cp $lib mpcium_amd/libmpcx_host.so.tmp && mv mpcium_amd/libmpcx_host.so.tmp mpcium_amd/libmpcx_host.so
  MPCX_HOST_TRACE=$O/host_$tag.csv MPCX_KTRACE=$O/k_$tag.csv timeout -k 10 300 python3 bench.py --detail $O/d_$tag.json --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline --no-sign3 > $O/l_$tag.json 2> $O/e_$tag.txt
  rc=$?
  cp $O/orig.so mpcium_amd/libmpcx_host.so
  [ $rc -eq 0 ] || { tail $O/e_$tag.txt; exit 1; }
  python3 tools/timeline.py $O/host_$tag.csv $O/k_$tag.csv $tag > $O/tl_$tag.json && head -40 $O/tl_$tag.json
done
