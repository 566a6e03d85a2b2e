"""CPU tests of the drop-in library's process lifecycle.

* The background start-up (csrc/rle_dropin.cpp preinit_*) starts only in a program that links the
  library (the reference server, linked by e2e/Makefile as INTEGRATION.md §2 shows), or when
  RLE_MI355X_PREINIT > 0: loading the library from Python does no GPU work before the first call.
* The start-up thread, its context pool, the pthread-key destructors, fork and the exit ordering run
  under AddressSanitizer and ThreadSanitizer builds of the drop-in (make lifecycle) with
  RLE_MI355X_FAKE_DEVICES, so no GPU is needed; tests/native/lifecycle_driver.c drives the
  reference server's own lifecycle: worker threads (/root/reference/src/server.c:520-524) and exit
  with workers still running (:615-623).  r4a's heap corruption (a pool re-initialised under the
  running start-up thread) was of this class.
"""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "c-filestorage-server-and-client_amd")
DRIVER = os.path.join(REPO, "tests", "native", "lifecycle_driver.c")

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None, reason="needs gcc/g++")


def _run(cmd, env=None, timeout=120):
    e = dict(os.environ)
    e.pop("RLE_MI355X_PREINIT", None)
    e.update(env or {})
    return subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=timeout)


def test_python_load_starts_no_gpu_work():
    """ctypes-loading the product library (as rle_mi355x.py, bench.py and the tests do) starts no
    background thread: rle_mi355x_preinit_state() is 0 until asked for with RLE_MI355X_PREINIT."""
    code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); print(L.rle_mi355x_preinit_state())")
    lib = os.path.join(PKG, "librle_mi355x.so")
    r = _run([sys.executable, "-c", code, lib])
    assert r.returncode == 0 and r.stdout.strip() == "0", (r.stdout, r.stderr[-2000:])
    r = _run([sys.executable, "-c", code, lib], {"RLE_MI355X_PREINIT": "2"})
    assert r.returncode == 0 and r.stdout.strip() == "1", (r.stdout, r.stderr[-2000:])


def test_linked_program_starts_up_in_background(tmp_path):
    """A C program linked against librle_mi355x.so (DT_NEEDED, like the reference server) gets the
    start-up by default (its main() waits, bounded, for phase 1; without a GPU that ends at once);
    RLE_MI355X_PREINIT=0 turns it off."""
    src = tmp_path / "pi.c"
    src.write_text("#include <stdio.h>\nint rle_mi355x_preinit_state(void);\n"
                   "int main(void){printf(\"%d\\n\", rle_mi355x_preinit_state());return 0;}\n")
    exe = tmp_path / "pi"
    subprocess.run(["gcc", str(src), "-o", str(exe), "-L" + PKG, "-lrle_mi355x", "-Wl,-rpath," + PKG], check=True)
    r = _run([str(exe)])
    assert r.returncode == 0 and r.stdout.strip() == "1", (r.stdout, r.stderr[-2000:])
    r = _run([str(exe)], {"RLE_MI355X_PREINIT": "0"})
    assert r.returncode == 0 and r.stdout.strip() == "0", (r.stdout, r.stderr[-2000:])


@pytest.fixture(scope="module")
def lifecycle_builds(tmp_path_factory):
    d = tmp_path_factory.mktemp("lc")
    LC = str(d)   # (the sanitizer builds stay out of the tree: nothing on the GPU box needs them)
    subprocess.run(["make", "-s", "-C", PKG, "lifecycle", "LCDIR=" + LC], check=True, capture_output=True, timeout=900)
    exes = {}
    for san, flag in (("asan", "address"), ("tsan", "thread")):
        lib = f"rle_mi355x_lc_{san}"
        exe = str(d / f"lc_{san}")
        subprocess.run(["gcc", "-O1", "-g", f"-fsanitize={flag}", "-pthread", DRIVER, "-o", exe, "-L" + LC, "-l" + lib,
                        "-Wl,-rpath," + LC], check=True)
        exed = str(d / f"lcd_{san}")
        subprocess.run(["gcc", "-O1", "-g", f"-fsanitize={flag}", "-pthread", "-DLC_DLOPEN", DRIVER, "-o", exed, "-ldl"],
                       check=True)
        exes[san] = (exe, exed, os.path.join(LC, f"lib{lib}.so"))
    return exes


@pytest.mark.parametrize("san", ["asan", "tsan"])
@pytest.mark.parametrize("scenario", ["exit", "exit_nowait", "workers", "fork", "fork_nowait", "dlopen"])
def test_lifecycle_under_sanitizers(lifecycle_builds, san, scenario):
    """Immediate exit (after the constructor's wait for phase 1, and with RLE_MI355X_PREINIT_WAIT_MS=0
    while the start-up thread is still building contexts); exit while worker threads are still in
    their key destructors; fork during start-up (the child must not wait for a start-up that has no
    thread in it); dlopen after main with RLE_MI355X_PREINIT=8.  Each must exit 0 with no sanitizer
    report."""
    exe, exed, lib = lifecycle_builds[san]
    env = {"RLE_MI355X_FAKE_DEVICES": "2", "RLE_MI355X_FAKE_DELAY_US": "5000",
           "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0", "TSAN_OPTIONS": "halt_on_error=1"}
    if scenario.endswith("_nowait"):
        env["RLE_MI355X_PREINIT_WAIT_MS"] = "0"
        scenario = scenario[:-len("_nowait")]
    if scenario == "dlopen":
        env["RLE_MI355X_PREINIT"] = "8"
        r = _run([exed, "dlopen", lib], env)
    else:
        r = _run([exe, scenario], env)
    report = [l for l in r.stderr.splitlines() if "Sanitizer" in l or "WARNING: ThreadSanitizer" in l]
    assert r.returncode == 0 and not report, (r.returncode, r.stderr[-4000:])
