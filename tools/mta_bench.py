"""Quick config-4 probe: MtA work of 2-of-3 signing for W wallets (GPU)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpcium_amd import host, mta, mpcx
mpcx.init(0); host.init(0)
d = json.load(open("tests/golden/node_preparams.json"))
nodes = [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]
for wallets in [int(x) for x in (sys.argv[1:] or ["64", "1000", "4000"])]:
    for signers in (2,):
        st = mta.bench_signing_mta(nodes, signers, wallets)
        st["sigs_per_s"] = wallets / st["total_s"]
        print(json.dumps({"signers": signers, **st}), flush=True)
