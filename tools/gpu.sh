# One parameterised GPU-box script (replaces round 2's one-off tools/gpu_*.sh).
# Every GPU step runs under its own time limit; steps chain with && so the
# first failure (fault, abort, timeout) ends the call.
#
#   bash tools/gpu.sh suite  OUT                 pytest -m gpu + smoke
#   bash tools/gpu.sh bench  OUT [bench args]    bench.py -> OUT/bench.json + summary
#   bash tools/gpu.sh trace  OUT [bench args]    rocprofv3 --kernel-trace --stats of bench.py + segments
#   bash tools/gpu.sh pmc    OUT COUNTERS [bench args]   one rocprofv3 --pmc pass (COUNTERS comma-free, space-joined in quotes)
#   bash tools/gpu.sh ab     OUT N LIB_A LIB_B [bench args]  N interleaved config-2 runs per libmpcx build
#   bash tools/gpu.sh abswap OUT N LIB_A LIB_B [bench args]  N interleaved full-bench runs, LIB swapped in place
#   bash tools/gpu.sh abhost OUT N HOSTLIB_A,HOSTLIB_B [bench args]  N interleaved runs per libmpcx_host build
#   bash tools/gpu.sh envab  OUT N "ENV_A" "ENV_B" [bench args]  N interleaved runs under two environments
#   bash tools/gpu.sh envn   OUT N "ENV1;ENV2;..." [bench args]  N interleaved runs per environment
#   bash tools/gpu.sh argab  OUT N "ARGS_A" "ARGS_B" [bench args]  N interleaved runs with two bench.py argument sets
#   bash tools/gpu.sh py     OUT script.py [args]            any python tool (tools/*.py) under a 600 s limit
set -o pipefail
mode=$1; O=gpurun_out/$2; shift 2
mkdir -p $O && export TMPDIR=/tmp
summ() {
python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
short = len(sys.argv) > 2 and sys.argv[2] == "short"
r = d["roofline"]
print("config2", round(d["value"]), "frac", round(r["frac"], 4), "kernel_ms", round(r["kernel_ms"], 2),
      "digest", d.get("batch_digest", {}).get("match"), "steps", d.get("step_kernel_ms", {}).get("per_step"))
if short:
    sys.exit(0)
t = d.get("gpu_telemetry") or {}
for k, v in t.items():
    if isinstance(v, dict) and any(s in k for s in ("gfxclk", "socket_power", "hotspot")):
        print("  telemetry", k, {a: round(b, 1) for a, b in v.items()})
for s in d.get("config2_per_operand_exponents", []):
    print("  per-operand", s["exp_bits"], round(s["value"]), round(s["kernel_ms"], 2), round(s["roofline"]["frac"], 3))
for k in ("signing", "signing_3_signers", "keygen", "safe_prime", "paillier_batch"):
    s = d.get(k)
    if s:
        print(k, round(s["value"], 1), s.get("unit"), "frac", (s.get("roofline") or {}).get("frac"),
              "cpu", (s.get("cpu_baseline") or {}).get("value"), "host_cpu_s", s.get("host_cpu_s"))
EOF
}
case $mode in
suite)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
  rc=$?; tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu.txt | head -20; exit 1; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
  tail -2 $O/smoke.txt ;;
bench)
  timeout -k 10 900 python3 bench.py --detail $O/bench_detail.json "$@" > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  wc -c $O/bench.json; summ $O/bench_detail.json ;;
trace)
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py \
      --detail $O/bench_detail.json "$@" > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  summ $O/bench_detail.json
  f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_segments.py $f > $O/trace_segments.txt && head -60 $O/trace_segments.txt
  find $O/prof -name '*kernel_stats*' -exec cp {} $O/kernel_stats.csv \; ;;
pmc)
  ctr=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/prof -o pmc -- python3 bench.py --detail $O/bench_detail.json "$@" \
      > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; } ;;
ab)
  n=$1; la=$2; lb=$3; shift 3
  for i in $(seq 1 $n); do
    for lib in $la $lb; do
      [ $lib = $la ] && tag=A_$i || tag=B_$i
      MPCX_LIB_PATH=$(realpath $lib) timeout -k 10 300 python3 bench.py --detail $O/ab_$tag.json "$@" > $O/ab_$tag.line \
          2> $O/ab_$tag.err || { tail $O/ab_$tag.err; exit 1; }
      echo -n "$lib run $i: "; summ $O/ab_$tag.json short
    done
  done ;;
abswap)
  # whole-library A/B: the variant replaces mpcium_amd/libmpcx.so for its runs
  # (libmpcx_host.so loads that file), the original is restored after each
  n=$1; la=$2; lb=$3; shift 3
  cp mpcium_amd/libmpcx.so $O/orig_libmpcx.so
  for i in $(seq 1 $n); do
    for lib in $la $lb; do
      [ $lib = $la ] && tag=A_$i || tag=B_$i
      cp $lib mpcium_amd/libmpcx.so.tmp && mv mpcium_amd/libmpcx.so.tmp mpcium_amd/libmpcx.so
      timeout -k 10 600 python3 bench.py --detail $O/ab_$tag.json "$@" > $O/ab_$tag.line 2> $O/ab_$tag.err
      rc=$?
      cp $O/orig_libmpcx.so mpcium_amd/libmpcx.so
      [ $rc -eq 0 ] || { tail $O/ab_$tag.err; exit 1; }
      echo "== $lib run $i"; summ $O/ab_$tag.json
    done
  done
  rm -f $O/orig_libmpcx.so ;;
abn)
  # like abswap for any number of builds (comma-separated); tag = position in the list
  n=$1; libs=$2; shift 2
  cp mpcium_amd/libmpcx.so $O/orig_libmpcx.so
  for i in $(seq 1 $n); do
    k=0
    for lib in ${libs//,/ }; do
      k=$((k+1)); tag=L${k}_$i
      cp $lib mpcium_amd/libmpcx.so.tmp && mv mpcium_amd/libmpcx.so.tmp mpcium_amd/libmpcx.so
      timeout -k 10 600 python3 bench.py --detail $O/ab_$tag.json "$@" > $O/ab_$tag.line 2> $O/ab_$tag.err
      rc=$?
      cp $O/orig_libmpcx.so mpcium_amd/libmpcx.so
      [ $rc -eq 0 ] || { tail $O/ab_$tag.err; exit 1; }
      echo "== $tag $lib"; summ $O/ab_$tag.json
    done
  done
  rm -f $O/orig_libmpcx.so ;;
abhost)
  # interleaved full-bench runs over host-library builds (comma-separated; see
  # tools/build_host_variant.sh): each replaces mpcium_amd/libmpcx_host.so for its run
  n=$1; libs=$2; shift 2
  cp mpcium_amd/libmpcx_host.so $O/orig_libmpcx_host.so
  for i in $(seq 1 $n); do
    k=0
    for lib in ${libs//,/ }; do
      k=$((k+1)); tag=H${k}_$i
      cp $lib mpcium_amd/libmpcx_host.so.tmp && mv mpcium_amd/libmpcx_host.so.tmp mpcium_amd/libmpcx_host.so
      timeout -k 10 600 python3 bench.py --detail $O/ab_$tag.json "$@" > $O/ab_$tag.line 2> $O/ab_$tag.err
      rc=$?
      cp $O/orig_libmpcx_host.so mpcium_amd/libmpcx_host.so
      [ $rc -eq 0 ] || { tail $O/ab_$tag.err; exit 1; }
      echo "== $tag $lib"; summ $O/ab_$tag.json
    done
  done
  rm -f $O/orig_libmpcx_host.so ;;
envab)
  n=$1; ea=$2; eb=$3; shift 3
  for i in $(seq 1 $n); do
    for e in A B; do
      [ $e = A ] && ev="$ea" || ev="$eb"
      env $ev timeout -k 10 600 python3 bench.py --detail $O/ab_${e}_$i.json "$@" > $O/ab_${e}_$i.line 2> $O/ab_${e}_$i.err \
          || { tail $O/ab_${e}_$i.err; exit 1; }
      echo "== $e ($ev) run $i"; summ $O/ab_${e}_$i.json
    done
  done ;;
envn)
  # N interleaved runs over several environments (separated by ';'), tag E<k>
  n=$1; envs=$2; shift 2
  IFS=';' read -ra EV <<< "$envs"
  for i in $(seq 1 $n); do
    k=0
    for ev in "${EV[@]}"; do
      k=$((k+1)); tag=E${k}_$i
      env $ev timeout -k 10 600 python3 bench.py --detail $O/ab_$tag.json "$@" > $O/ab_$tag.line 2> $O/ab_$tag.err \
          || { tail $O/ab_$tag.err; exit 1; }
      echo "== $tag ($ev)"; summ $O/ab_$tag.json short
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('  ', {k: round(d[k]['value'],1) for k in ('signing','signing_3_signers','keygen','paillier_batch') if k in d})" $O/ab_$tag.json
    done
  done ;;
argab)
  # N interleaved runs of bench.py with two extra-argument strings A and B (same build)
  n=$1; aa=$2; ab=$3; shift 3
  for i in $(seq 1 $n); do
    for e in A B; do
      [ $e = A ] && ex="$aa" || ex="$ab"
      timeout -k 10 600 python3 bench.py --detail $O/ab_${e}_$i.json $ex "$@" > $O/ab_${e}_$i.line 2> $O/ab_${e}_$i.err \
          || { tail $O/ab_${e}_$i.err; exit 1; }
      echo "== $e ($ex) run $i"; summ $O/ab_${e}_$i.json
    done
  done ;;
py)
  timeout -k 10 600 python3 -u "$@" > $O/out.txt 2> $O/err.txt || { tail -20 $O/err.txt; tail -20 $O/out.txt; exit 1; }
  tail -40 $O/out.txt ;;
*) echo "unknown mode $mode"; exit 2 ;;
esac
