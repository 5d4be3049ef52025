"""GPU tests of the one-process-many-GPUs boundary (include/mpcx.h
mpcx_init_devices / mpcx_select_device / mpcx_modexp_submit): every visible
GPU bound in this process (one on the test box), batches split by the
partition plan with forced small slices, asynchronous jobs, and two
device-buffer calls on different streams in flight at once (each stream has
its own workspace)."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx(gpu):
    from mpcium_amd import mpcx
    mpcx.init_devices(0)
    return mpcx


def _key():
    k = load_golden("paillier_key_2048.json")
    return int(k["N"], 16)


def test_bound_devices(mx):
    devs = mx.bound_devices()
    assert len(devs) == mx.device_count() and devs == list(range(len(devs)))
    mx.select_device(0)
    with pytest.raises(mx.MpcxError):
        mx.select_device(len(devs))


def test_split_batches_match_pow(mx):
    """Small device_split_min forces multi-slice plans (one slice per bound
    device); results are gathered in operand order."""
    import random
    N = _key()
    N2 = N * N
    rng = random.Random(5)
    mod = mx.Modulus(N2)
    try:
        xs = [rng.randrange(N2) for _ in range(97)]
        es = [rng.getrandbits(rng.choice([64, 256, 700])) for _ in range(97)]
        mx.set_option("device_split_min", 8)
        try:
            got = mod.exp(xs, es)
            got_shared = mod.exp(xs, N)
        finally:
            mx.set_option("device_split_min", 4096)
        assert got == [pow(x, e, N2) for x, e in zip(xs, es)]
        assert got_shared == [pow(x, N, N2) for x in xs]
    finally:
        mod.release()


def test_async_jobs(mx):
    import random
    N = _key()
    rng = random.Random(6)
    mod = mx.Modulus(N)
    try:
        batches = [[rng.randrange(N) for _ in range(50 + 13 * i)] for i in range(4)]
        jobs = [mod.submit(b, N - 1 - i) for i, b in enumerate(batches)]
        for i, (b, j) in enumerate(zip(batches, jobs)):
            assert j.wait() == [pow(x, N - 1 - i, N) for x in b]
    finally:
        mod.release()


def test_device_buffers_on_two_streams(mx):
    """Two asynchronous device-buffer batches with different shared
    exponents on two streams: each stream's schedule and window tables live in
    its own workspace (a single shared workspace raced here)."""
    import ctypes
    N = _key()
    mod = mx.Modulus(N)
    L = mx.lib()
    try:
        count, w = 4096, mod.class_words
        rng = np.random.default_rng(9)
        host = rng.integers(0, 1 << 32, size=(count, w), dtype=np.uint64).astype(np.uint32)
        host[:, -1] = 0
        host[:, (N.bit_length() - 1) // 32:] = 0
        e1, e2 = N, (N - 1) // 2
        E1, E2 = mx.int_to_words(e1, mx.nwords(e1)), mx.int_to_words(e2, mx.nwords(e2))
        ptr = {}
        for name, nbytes in (("b", host.nbytes), ("e1", E1.nbytes), ("e2", E2.nbytes), ("o1", count * w * 4),
                             ("o2", count * w * 4)):
            p = ctypes.c_void_p()
            mx._check(L.mpcx_dev_alloc(nbytes, ctypes.byref(p)))
            ptr[name] = p
        s1, s2 = ctypes.c_void_p(), ctypes.c_void_p()
        mx._check(L.mpcx_stream_create(ctypes.byref(s1)))
        mx._check(L.mpcx_stream_create(ctypes.byref(s2)))
        try:
            mx._check(L.mpcx_memcpy_h2d(ptr["b"], host.ctypes.data, host.nbytes))
            mx._check(L.mpcx_memcpy_h2d(ptr["e1"], E1.ctypes.data, E1.nbytes))
            mx._check(L.mpcx_memcpy_h2d(ptr["e2"], E2.ctypes.data, E2.nbytes))
            for _ in range(2):
                mx._check(L.mpcx_modexp_batch_device(mod.handle, count, ptr["b"], w, ptr["e1"], len(E1), 1,
                                                     e1.bit_length(), ptr["o1"], w, s1))
                mx._check(L.mpcx_modexp_batch_device(mod.handle, count, ptr["b"], w, ptr["e2"], len(E2), 1,
                                                     e2.bit_length(), ptr["o2"], w, s2))
            mx._check(L.mpcx_sync(s1))
            mx._check(L.mpcx_sync(s2))
            o1 = np.zeros((count, w), dtype="<u4")
            o2 = np.zeros((count, w), dtype="<u4")
            mx._check(L.mpcx_memcpy_d2h(o1.ctypes.data, ptr["o1"], o1.nbytes))
            mx._check(L.mpcx_memcpy_d2h(o2.ctypes.data, ptr["o2"], o2.nbytes))
        finally:
            mx._check(L.mpcx_stream_destroy(s1))
            mx._check(L.mpcx_stream_destroy(s2))
            for p in ptr.values():
                L.mpcx_dev_free(p)
        xs = mx.words_to_ints(host)
        r1, r2 = mx.words_to_ints(o1), mx.words_to_ints(o2)
        for i in range(0, count, 97):
            assert r1[i] == pow(xs[i], e1, N) and r2[i] == pow(xs[i], e2, N), i
    finally:
        mod.release()


_LOGICAL = r"""
import json, random, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
from conftest import load_golden
from mpcium_amd import host, mpcx, mta, proofs
mpcx.set_option("duplicate_device", 1)
host.init(0)
host.init(0)
out = {"devices": mpcx.bound_devices()}
N = int(load_golden("paillier_key_2048.json")["N"], 16)
N2 = N * N
rng = random.Random(11)
mod = mpcx.Modulus(N2)
xs = [rng.randrange(N2) for _ in range(300)]
mpcx.set_option("device_split_min", 64)
l0 = [mpcx.device_launches(i) for i in range(2)]
out["split_ok"] = mod.exp(xs, N) == [pow(x, N, N2) for x in xs]
out["split_launches"] = [mpcx.device_launches(i) - l0[i] for i in range(2)]
# the matrix-core kernel on both logical devices: each builds and uploads its own tables
mpcx.set_option("device_split_min", 2048)
mpcx.set_option("geom_policy", 2)
mpcx.set_option("kernel_stats", 1)
mpcx.kernel_stats(reset=True)
ys = [rng.randrange(N2) for _ in range(4160)]
l0 = [mpcx.device_launches(i) for i in range(2)]
got = mod.exp(ys, N)
ks = mpcx.kernel_stats()
out["mx_split_ok"] = all(got[i] == pow(ys[i], N, N2) for i in rng.sample(range(len(ys)), 24))
out["mx_split_launches"] = [mpcx.device_launches(i) - l0[i] for i in range(2)]
out["mx_operands"] = sum(k["operands"] for k in ks["kernels"] if k["kind"] == "modexp_mx")
mpcx.set_option("kernel_stats", 0)
mpcx.set_option("geom_policy", 1)
mod.release()
mpcx.set_option("device_split_min", 4096)
d = load_golden("node_preparams.json")
nodes = [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]
l1 = [mpcx.device_launches(i) for i in range(2)]
out["signing"] = mta.bench_signing(nodes, 2, 300, seed=0x10D)
out["keygen"] = proofs.bench_keygen_proofs(nodes, 24, seed=0x10E, wave=12)
out["work_launches"] = [mpcx.device_launches(i) - l1[i] for i in range(2)]
print(json.dumps(out))
"""


def test_two_logical_devices(gpu):
    """One HIP ordinal bound twice (mpcx_set_option "duplicate_device", a test
    hook) in a child process: a split batch runs one slice per logical device
    concurrently and gathers in order, and the signing and keygen drivers
    spread their batches over both devices' lanes -- the one-process-many-GPUs
    node shape (/root/reference/pkg/mpc/node.go:69,109) exercised on one GPU."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _LOGICAL, root], capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["devices"] == [0, 0]
    assert out["split_ok"] and all(n >= 1 for n in out["split_launches"])
    assert out["mx_split_ok"] and all(n >= 1 for n in out["mx_split_launches"]) and out["mx_operands"] == 4160
    s = out["signing"]
    assert s["errors"] == 0 and s["relation_failures"] == 0 and s["verified"] == 300 and s["aborted"] == 0
    assert out["keygen"]["failures"] == 0 and out["keygen"]["waves"] == 2
    assert all(n > 0 for n in out["work_launches"]), out["work_launches"]


def test_bench_two_ranks(gpu, tmp_path):
    """The driver's N-GPU bench path end to end, at small sizes: `bench.py
    --gpus 2` without a launcher re-launches itself under torchrun (two ranks;
    LOCAL_RANK wraps onto this box's GPU), every rank runs its own config-2
    batch (checked against pow on a sample inside bench.py), signing wallets,
    config-1 batches and config-5 sessions, the safe-prime search is sharded,
    and rank 0 prints ONE parseable line with n_gpus 2 and every config."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    detail = tmp_path / "detail.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--count", "4096", "--wallets", "300", "--keygen-sessions", "64", "--keygen-wave", "32",
           "--safe-primes", "8", "--no-cpu-baseline", "--no-smi", "--detail", str(detail)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert len(lines[0]) <= 4096
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    for k in ("c1_paillier", "c3_safe_primes", "c4_sign", "c4_sign_3_signers", "c5_keygen"):
        assert line["configs"][k]["n_gpus"] == 2, k
        assert line["configs"][k]["value"] > 0, k
    full = json.load(open(detail))
    assert full["signing"]["signatures_verified"] == 600
    assert full["keygen"]["sessions"] == 64


def test_bench_node_mode(gpu, tmp_path):
    """`bench.py --node`: mpcium's one-process-per-node shape
    (/root/reference/pkg/mpc/node.go:59-88) -- one process binds the node's
    devices (here one HIP ordinal bound twice, the rehearsal hook) and runs
    config 2 (one resident batch per device, device 0's whole batch checked
    against the C restatement's digest, every device sampled against pow),
    config 4 and config 5 through the one Engine: every device receives
    launches in every config, and one parseable line reports mode "node"."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    detail = tmp_path / "node.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--node", "--node-dup", "2", "--steps", "1",
           "--warmup", "1", "--count", "65536", "--wallets", "300", "--keygen-sessions", "64", "--keygen-wave", "32",
           "--detail", str(detail)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["mode"] == "node" and line["n_gpus"] == 2 and line["value"] > 0
    assert line["digest_match"] is True
    assert all(n > 0 for n in line["device_launches"]), line["device_launches"]
    for k in ("c4_sign", "c5_keygen"):
        assert line["configs"][k]["value"] > 0
        assert all(n > 0 for n in line["configs"][k]["device_launches"]), (k, line["configs"][k])
    full = json.load(open(detail))
    assert full["signing"]["signatures_verified"] == 600
    assert full["keygen"]["sessions"] == 128 and full["keygen"]["reshare_sessions"] > 0
