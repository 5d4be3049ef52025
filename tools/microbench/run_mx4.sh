# timing split (product alone / reduction alone / full) and PMC of the LDS-table chain kernel
set -o pipefail
O=gpurun_out/mx4; mkdir -p $O
cd tools/microbench
for v in t1 t2; do MX_CHAIN_SO=mx_chain_$v.so timeout -k 10 120 python -u mx_chain.py 65536 64 > ../../$O/chain_$v.json 2>/dev/null || exit 1; done
timeout -k 10 120 python -u mx_chain.py 65536 64 > ../../$O/chain_full.json 2>/dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d ../../$O/a -o pmc -- python3 mx_chain.py 65536 64 > ../../$O/a.json 2> ../../$O/a.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_MFMA --output-format csv -d ../../$O/b -o pmc -- python3 mx_chain.py 65536 64 > ../../$O/b.json 2> ../../$O/b.err || exit 1
cd ../..
cat $O/chain_*.json
for f in $(find $O -name '*counter_collection.csv'); do python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r.get("Kernel_Name", "")[:14]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if "chain" in k:
        print(k, {c: round(x) for c, x in sorted(v.items())})
PY
done
