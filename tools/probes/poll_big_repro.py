#!/usr/bin/env python3
"""Diagnosis of a one-off 'dec-big' mismatch of tests/test_gpu_hostpath.py::test_polled_small_calls
(RLE_MI355X_ZC_SEG=8192, a registered decompress with an extra region after 640 zero-copy calls):
runs that test's own code several times in fresh processes with the mismatching bytes reported.
usage: python tools/probes/poll_big_repro.py [runs] [repetitions of the body per run]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "tests", "test_gpu_hostpath.py")).read()
code = re.search(r"_POLL_CODE = r'''(.*?)'''", src, re.S).group(1)
diag = '''
        got = R.decompress(y, U, E)
        want = x + bytes(E)
        i = next((j for j in range(len(want)) if got[j] != want[j]), -1)   # (-1: the repeat matched)
        nz = sum(1 for j in range(0, len(want), 4096) if got[j:j + 4096] == bytes(len(got[j:j + 4096])))
        print("MISMATCH", k, U, E, len(y), "first", i, got[i:i + 8].hex(), want[i:i + 8].hex(),
              "zero-pages", nz, (len(want) + 4095) // 4096, "stats", R.dropin_stats(), flush=True)
        errors.append(("dec-big", k, U, E))'''
code = code.replace('''        errors.append(("dec-big", k, U, E))''', diag.lstrip("\n"), 1)
# the test's body repeated in one process (its allocation pattern, many times over)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
if reps > 1:
    head, body = code.split("errors = []", 1)
    body, tail = body.split("def work(t):", 1)
    body = "\n".join("    " + l for l in body.splitlines())
    code = head + "errors = []\nfor _rep in range(%d):\n" % reps + body + "\ndef work(t):" + tail
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
bad = 0
for r in range(runs):
    env = dict(os.environ, RLE_MI355X_POLL="1", RLE_MI355X_SERVICE="0", RLE_MI355X_ZC_SEG="8192")
    p = subprocess.run([sys.executable, "-c", code, os.path.join(ROOT, "c-filestorage-server-and-client_amd"),
                        os.path.join(ROOT, "oracle")], env=env, capture_output=True, text=True, timeout=400)
    print("run", r, "rc", p.returncode, p.stdout[-3000:], p.stderr[-1500:], flush=True)
    bad += p.returncode != 0
sys.exit(1 if bad else 0)
