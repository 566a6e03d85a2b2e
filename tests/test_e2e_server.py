"""End-to-end: the UNCHANGED reference server and client over their AF_UNIX socket, with the
reference codec (server_ref, BASELINE configs[0]) and with librle_mi355x.so linked in its place
(server_gpu, configs[4]); binaries from e2e/Makefile (built from /root/reference).

Battery 1 follows tests/test1.sh:13,17 (write file1,file2 and read them back; write the rec
directory and read everything back with -R 0) and checks what the reference's script never
does: every returned file is byte-identical to its source, and the server's exit statistic
"Max total storage size reached" is 363500 bytes (the sum of the compressed sizes).
Battery 2 follows tests/test2.sh:6-30 (LRU eviction with MAXSTORAGECAP=1000000): big2 + randbig
fit (942363 compressed bytes), writing big4 evicts randbig, which is decoded and shipped back
(src/server.c:312-323) and must match its source.
Battery LFU follows tests/test2.sh:36-64 (REPLACEMENTALGO=2): randbig read twice and big2 once, so
writing big4 evicts big2, the least frequently used.  Battery victims follows tests/test2.sh:70-88:
writing big1 (333334 compressed bytes) next to big2 + randbig evicts both.  Each checks the shipped
files byte for byte and the server's exit statistics (max storage, files evicted).
Battery concurrent follows the shape of tests/test3.sh (WORKERPOOLSIZE=8, several clients at once;
the script's bigfiles/biggest* inputs are absent from the reference, .MISSING_LARGE_BLOBS): 8
clients each write their own directory of 24 files (4-40 KiB random / zero / run-heavy, and the
reference's smallfiles/small1, small7) and read every file back, all at once; every returned file
must be byte-identical to its source.
"""
import json
import os
import re
import shutil
import signal
import subprocess
import time

import pytest

from conftest import GOLDEN, REPO

BIN = os.path.join(REPO, "e2e", "_bin")
CLIENT = os.path.join(BIN, "client")
ANSI = re.compile(r"\x1b\[[0-9;]*m")


def _need(exe):
    if not (os.path.exists(exe) and os.path.exists(CLIENT)):
        pytest.skip(f"{exe} not built (make -C e2e needs /root/reference)")


def _stage_files(tmp):
    d = os.path.join(tmp, "files")
    for rel in ("file1", "file2", "rec/rec1", "rec/rec2", "bigfiles/randbig"):
        dst = os.path.join(d, rel)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copyfile(os.path.join(GOLDEN, "dummyFiles", rel.replace("/", "__")), dst)
    for rel, U in (("bigfiles/big2", 360000), ("bigfiles/big4", 360000), ("bigfiles/big1", 1000000)):
        with open(os.path.join(d, rel), "wb") as f:
            f.write(bytes(U))
    return d


class Server:
    """settle: seconds to wait after the socket appears (a server that has been up for a moment:
    the drop-in's background start-up, csrc/rle_dropin.cpp preinit_main, has run)."""

    def __init__(self, exe, tmp, cfg, env=None, settle=0.0):
        self.tmp = tmp
        self.sock = os.path.join(tmp, "s.sk")
        conf = dict(cfg, SOCKETFILENAME=self.sock, LOGFILENAME=os.path.join(tmp, "logs.json"))
        path = os.path.join(tmp, "config.txt")
        with open(path, "w") as f:
            f.write("".join(f"{k}={v}\n" for k, v in conf.items()))
        self.p = subprocess.Popen([exe, path], cwd=tmp, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                  env=dict(os.environ, **(env or {})))
        t0 = time.time()
        while not os.path.exists(self.sock):
            if self.p.poll() is not None or time.time() - t0 > 60:
                raise RuntimeError("server did not start: " + self.p.stdout.read().decode(errors="replace"))
            time.sleep(0.005)
        self.startup_s = time.time() - t0   # spawn -> socket (the drop-in's start-up runs before main)
        if settle:
            time.sleep(settle)

    def client(self, *args):
        r = subprocess.run([CLIENT, "-f", self.sock, "-t", "0", *args], cwd=self.tmp, capture_output=True,
                           timeout=120)
        assert r.returncode == 0, (args, r.stdout.decode(errors="replace"), r.stderr.decode(errors="replace"))
        return r

    def stop(self):
        self.p.send_signal(signal.SIGHUP)
        out, _ = self.p.communicate(timeout=120)
        return ANSI.sub("", out.decode(errors="replace"))


def _max_storage(text):
    m = re.search(r"Max total storage size reached: (\d+) bytes", text)
    assert m, text[-2000:]
    return int(m.group(1))


def _victims(text):
    m = re.search(r"Number of files that have been evicted from the cache: (\d+)", text)
    assert m, text[-2000:]
    return int(m.group(1))


def _returned(root):
    out = {}
    for d, _, fs in os.walk(root):
        for fn in fs:
            out.setdefault(fn, []).append(open(os.path.join(d, fn), "rb").read())
    return out


def battery1(exe, tmp, env=None, settle=0.0):
    files = _stage_files(tmp)
    srv = Server(exe, tmp, {"MAXSTORAGECAP": 128000000, "MAXFILECOUNT": 10000, "WORKERPOOLSIZE": 1}, env, settle)
    t0 = time.perf_counter()
    try:
        f1, f2 = os.path.join(files, "file1"), os.path.join(files, "file2")
        srv.client("-W", f"{f1},{f2}", "-r", f"{f1},{f2}", "-d", os.path.join(tmp, "dest1"))
        srv.client("-w", f"{os.path.join(files, 'rec')},0", "-R", "0", "-d", os.path.join(tmp, "dest2"))
    finally:
        wall = time.perf_counter() - t0
        text = srv.stop()
    return _max_storage(text), _returned(os.path.join(tmp, "dest1")), _returned(os.path.join(tmp, "dest2")), wall


def battery2(exe, tmp, env=None, settle=0.0):
    files = _stage_files(tmp)
    srv = Server(exe, tmp, {"MAXSTORAGECAP": 1000000, "MAXFILECOUNT": 10, "WORKERPOOLSIZE": 4,
                            "REPLACEMENTALGO": 1}, env, settle)
    b = lambda n: os.path.join(files, "bigfiles", n)
    t0 = time.perf_counter()
    try:
        srv.client("-W", f"{b('big2')},{b('randbig')}")
        time.sleep(1.1)   # the LRU clock has 1-second resolution (tests/test2.sh:18)
        srv.client("-r", b("big2"), "-d", os.path.join(tmp, "readback"))
        srv.client("-W", b("big4"), "-D", os.path.join(tmp, "evicted1"))
    finally:
        wall = time.perf_counter() - t0 - 1.1   # from the socket's appearance (+ settle), less the sleep
        text = srv.stop()
    return (_max_storage(text), _returned(os.path.join(tmp, "evicted1")), _returned(os.path.join(tmp, "readback")),
            wall)


def battery_lfu(exe, tmp, env=None):
    """tests/test2.sh:36-64: LFU (REPLACEMENTALGO=2); big2 is read once, randbig twice, so big4
    evicts big2."""
    files = _stage_files(tmp)
    srv = Server(exe, tmp, {"MAXSTORAGECAP": 1000000, "MAXFILECOUNT": 10, "WORKERPOOLSIZE": 4,
                            "REPLACEMENTALGO": 2}, env)
    b = lambda n: os.path.join(files, "bigfiles", n)
    try:
        srv.client("-W", f"{b('big2')},{b('randbig')}")
        srv.client("-r", b("randbig"), "-d", os.path.join(tmp, "readback", "1"))
        srv.client("-r", b("randbig"), "-d", os.path.join(tmp, "readback", "2"))
        srv.client("-r", b("big2"), "-d", os.path.join(tmp, "readback", "3"))
        srv.client("-W", b("big4"), "-D", os.path.join(tmp, "evicted2"))
    finally:
        text = srv.stop()
    return _max_storage(text), _victims(text), _returned(os.path.join(tmp, "evicted2")), \
        _returned(os.path.join(tmp, "readback"))


def battery_victims(exe, tmp, env=None):
    """tests/test2.sh:70-88: big1 (C = 333334) does not fit next to big2 + randbig (942363 of
    1000000): both are evicted, decoded and shipped back in one write."""
    files = _stage_files(tmp)
    srv = Server(exe, tmp, {"MAXSTORAGECAP": 1000000, "MAXFILECOUNT": 10, "WORKERPOOLSIZE": 4,
                            "REPLACEMENTALGO": 2}, env)
    b = lambda n: os.path.join(files, "bigfiles", n)
    try:
        srv.client("-W", f"{b('big2')},{b('randbig')}")
        srv.client("-W", b("big1"), "-D", os.path.join(tmp, "evicted3"))
        srv.client("-r", b("big1"), "-d", os.path.join(tmp, "readback"))
    finally:
        text = srv.stop()
    return _max_storage(text), _victims(text), _returned(os.path.join(tmp, "evicted3")), \
        _returned(os.path.join(tmp, "readback"))


def _concurrent_files(tmp, c, nfiles, rnd):
    d = os.path.join(tmp, f"c{c}")
    os.makedirs(d, exist_ok=True)
    files = {}
    for k in range(nfiles):
        if k < 2:   # the reference's small files, once per client directory
            name = ("smallfiles__small1", "smallfiles__small7")[k]
            b = open(os.path.join(GOLDEN, "dummyFiles", name), "rb").read()
        else:
            U = rnd.choice([4096, 8192, 16384, 40000])
            kind = k % 3
            b = bytes(U) if kind == 1 else (rnd.randbytes(U) if kind == 0 else
                                            b"".join(bytes([rnd.randrange(256)]) * rnd.randrange(1, 12)
                                                     for _ in range(U // 4))[:U])
        p = os.path.join(d, f"f{c}_{k}")
        with open(p, "wb") as f:
            f.write(b)
        files[p] = b
    return d, files


def battery_concurrent(exe, tmp, env=None, clients=8, nfiles=24):
    """tests/test3.sh's shape: 8 workers, `clients` clients at once, each writing its directory (-w)
    and reading its files back (-r); returns {path: (source, [returned copies])}."""
    import random
    import threading
    rnd = random.Random(3)
    dirs = [_concurrent_files(os.path.join(tmp, "src"), c, nfiles, rnd) for c in range(clients)]
    srv = Server(exe, tmp, {"MAXSTORAGECAP": 512000000, "MAXFILECOUNT": 10000, "WORKERPOOLSIZE": 8}, env)
    errs = []

    def client(c, d, names):
        try:
            srv.client("-w", f"{d},0")
            srv.client("-r", ",".join(names), "-d", os.path.join(tmp, f"out{c}"))
        except Exception as e:   # noqa: BLE001 (reported below)
            errs.append(repr(e))

    try:
        th = [threading.Thread(target=client, args=(c, d, sorted(fs))) for c, (d, fs) in enumerate(dirs)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        text = srv.stop()
    assert not errs, errs[:3]
    got = {}
    for c in range(clients):
        got.update({k: v for k, v in _returned(os.path.join(tmp, f"out{c}")).items()})
    return {p: (b, got.get(os.path.basename(p), [])) for _, fs in dirs for p, b in fs.items()}, _max_storage(text)


def _check_lfu(res):
    stat, victims, ev, rb = res
    assert stat == 942363 and victims == 1
    assert list(ev) == ["big2"] and ev["big2"] == [bytes(360000)]
    assert rb["randbig"] == [_src("randbig")] * 2 and rb["big2"] == [bytes(360000)]


def _check_victims(res):
    stat, victims, ev, rb = res
    assert stat == 942363 and victims == 2
    assert sorted(ev) == ["big2", "randbig"]
    assert ev["big2"] == [bytes(360000)] and ev["randbig"] == [_src("randbig")]
    assert rb["big1"] == [bytes(1000000)]


def _check_concurrent(res):
    files, stat = res
    bad = [p for p, (b, copies) in files.items() if copies != [b]]
    assert not bad, (len(bad), bad[:3])
    assert stat == sum(len(O_encode(b)) for b, _ in files.values())


def O_encode(b):
    import rle_oracle as O
    return O.encode(b)


def _src(name):
    if name in ("big2", "big4"):
        return bytes(360000)
    if name == "big1":
        return bytes(1000000)
    rel = {"file1": "file1", "file2": "file2", "rec1": "rec/rec1", "rec2": "rec/rec2", "randbig": "bigfiles/randbig"}
    return open(os.path.join(GOLDEN, "dummyFiles", rel[name].replace("/", "__")), "rb").read()


def _check_battery1(res):
    stat, d1, d2, _ = res
    assert stat == 363500
    assert sorted(d1) == ["file1", "file2"] and sorted(d2) == ["file1", "file2", "rec1", "rec2"]
    for d in (d1, d2):
        for name, blobs in d.items():
            assert all(b == _src(name) for b in blobs), name


def _check_battery2(res):
    stat, ev, rb, _ = res
    assert stat == 942363
    assert list(ev) == ["randbig"] and ev["randbig"] == [_src("randbig")]
    assert rb["big2"] == [bytes(360000)]


def test_e2e_reference_server(tmp_path):
    exe = os.path.join(BIN, "server_ref")
    _need(exe)
    _check_battery1(battery1(exe, str(tmp_path / "b1")))
    _check_battery2(battery2(exe, str(tmp_path / "b2")))
    _check_lfu(battery_lfu(exe, str(tmp_path / "lfu")))
    _check_victims(battery_victims(exe, str(tmp_path / "victims")))
    _check_concurrent(battery_concurrent(exe, str(tmp_path / "conc")))


@pytest.mark.gpu
def test_e2e_gpu_server(tmp_path):
    exe = os.path.join(BIN, "server_gpu")
    _need(exe)
    stats = str(tmp_path / "dropin_stats.json")
    res1 = battery1(exe, str(tmp_path / "b1"), {"RLE_MI355X_STATS": stats})
    _check_battery1(res1)
    st = json.load(open(stats))
    assert st["calls_compress"] >= 4 and st["calls_decompress"] >= 6   # 4 writes; 6 reads
    _check_battery2(battery2(exe, str(tmp_path / "b2")))
    print("e2e gpu battery1 wall %.3fs dropin %s" % (res1[3], st))


@pytest.mark.gpu
def test_e2e_gpu_server_lfu_and_victims(tmp_path):
    """tests/test2.sh's LFU battery (:36-64) and multiple-victims battery (:70-88) against the
    drop-in: evicted files decoded on the GPU (src/server.c:317) and shipped back byte-identical."""
    exe = os.path.join(BIN, "server_gpu")
    _need(exe)
    _check_lfu(battery_lfu(exe, str(tmp_path / "lfu")))
    _check_victims(battery_victims(exe, str(tmp_path / "victims")))


@pytest.mark.gpu
def test_e2e_gpu_server_concurrent_workers(tmp_path):
    """tests/test3.sh's shape against the drop-in: 8 workers serving 8 clients at once, concurrent
    compress and decompress calls from the worker threads, every returned file byte-identical and
    the max-storage statistic equal to the oracle's compressed sizes."""
    exe = os.path.join(BIN, "server_gpu")
    _need(exe)
    _check_concurrent(battery_concurrent(exe, str(tmp_path / "conc")))
