#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ref/ from the REFERENCE itself.

Runs oracle/_ref/Application_replay -- the unmodified reference sources from
/root/reference compiled by oracle/Makefile with link-time hooks (oracle/ref_hooks.cpp) --
for the reference's three testcases x seeds x {glibc, philox} and stores, gzipped:

  dbg.log        the reference's event log            (Log.cpp:44-130)
  msgcount.log   per-node per-tick sent/recv counts   (EmulNet.cpp:184-220)
  state.txt      end-of-tick membership state of every node (ref_hooks.cpp format)
  stdout.txt     the driver's "i-th introduced node" lines (Application.cpp:146)

Only outputs (data) are committed; no reference source is copied.  Run from the repo root
in THIS container (the reference does not exist on the GPU box):

    make -C oracle ref && python tests/golden/make_golden.py
"""
import gzip
import hashlib
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.environ.get("GSP_REFERENCE", "/root/reference")
BIN = os.path.join(ROOT, "oracle", "_ref", "Application_replay")
OUT = os.path.join(ROOT, "tests", "golden", "ref")

CONFS = ["singlefailure", "multifailure", "msgdropsinglefailure"]
SEEDS = [1, 5, 9, 10, 1234567]
MODES = ["glibc", "philox"]


def run_one(conf, seed, mode, dest):
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "testcases"))
        src_conf = os.path.join(REF, "testcases", conf + ".conf")
        shutil.copy(src_conf, os.path.join(tmp, "testcases"))
        env = dict(os.environ, GSP_SEED=str(seed), GSP_RNG=mode,
                   GSP_STATE_DUMP=os.path.join(tmp, "state.txt"))
        out = subprocess.run([BIN, "testcases/%s.conf" % conf], cwd=tmp, env=env,
                             check=True, capture_output=True).stdout
        with open(os.path.join(tmp, "stdout.txt"), "wb") as f:
            f.write(out)
        os.makedirs(dest, exist_ok=True)
        for name in ["dbg.log", "msgcount.log", "state.txt", "stdout.txt"]:
            with open(os.path.join(tmp, name), "rb") as f, \
                    gzip.GzipFile(os.path.join(dest, name + ".gz"), "wb", mtime=0) as g:
                g.write(f.read())


# Beyond the reference's own N = 10 testcases (--big): our own .conf inputs at MAX_NNB 70, 300
# and 600 (the reference accepts up to MAX_NODES = 1000, EmulNet.h:10).  They reach the
# reference behaviour N = 10 never does: the msgcount.log line of node 67 (EmulNet.cpp:204-211),
# negative signed-char address bytes of ids >= 128 (Log.cpp:73), strcmp() aliasing of ids whose
# low byte is 0 -- 256 and 512 (EmulNet.cpp:154), the full 30,000-message buffer
# (EmulNet.cpp:92, reached once the multi-failure victims' messages linger) and the id < 10
# payload filter at N > 10 (MP1Node.cpp:245).  state.txt (tens of MB at N = 600) is stored as
# one SHA-256 per tick (state_sha.txt: "t hexdigest" of that tick's lines, each ending in \n)
# plus the full lines of a few ticks (state_sel.txt).
BIG_OUT = os.path.join(ROOT, "tests", "golden", "ref_big")
BIG_CONFS = {
    # name: (MAX_NNB, SINGLE_FAILURE, DROP_MSG)
    "n70_single": (70, 1, 0), "n70_multi": (70, 0, 0), "n70_drop": (70, 1, 1),
    "n300_single": (300, 1, 0), "n300_multi": (300, 0, 0), "n300_drop": (300, 1, 1),
    "n600_multidrop": (600, 0, 1), "n600_single": (600, 1, 0),
}
BIG_RUNS = [(c, s, m) for c in BIG_CONFS if not c.startswith("n600") for s in (3, 77)
            for m in MODES] + [(c, 3, m) for c in BIG_CONFS if c.startswith("n600") for m in MODES]
STATE_SEL = (99, 100, 101, 121, 299, 300, 699)


def state_digest(state_bytes):
    """(sha lines, selected lines) of a state dump: lines grouped by their tick field
    (tests/oracle_binding.state_digest is the same function, used by the parity tests)."""
    by_tick = {}
    for line in state_bytes.splitlines(keepends=True):
        by_tick.setdefault(int(line.split(b" ", 1)[0]), []).append(line)
    sha = b"".join(b"%d %s\n" % (t, hashlib.sha256(b"".join(v)).hexdigest().encode())
                   for t, v in sorted(by_tick.items()))
    sel = b"".join(b"".join(by_tick.get(t, [])) for t in STATE_SEL)
    return sha, sel


def write_big_conf(name):
    nnb, single, drop = BIG_CONFS[name]
    d = os.path.join(BIG_OUT, "testcases")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, name + ".conf"), "w") as f:
        f.write("MAX_NNB: %d\nSINGLE_FAILURE: %d\nDROP_MSG: %d\nMSG_DROP_PROB: 0.1\n"
                % (nnb, single, drop))


def run_big(conf, seed, mode):
    dest = os.path.join(BIG_OUT, mode, conf, str(seed))
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "testcases"))
        shutil.copy(os.path.join(BIG_OUT, "testcases", conf + ".conf"), os.path.join(tmp, "testcases"))
        env = dict(os.environ, GSP_SEED=str(seed), GSP_RNG=mode,
                   GSP_STATE_DUMP=os.path.join(tmp, "state.txt"))
        out = subprocess.run([BIN, "testcases/%s.conf" % conf], cwd=tmp, env=env,
                             check=True, capture_output=True).stdout
        files = {"stdout.txt": out}
        for name in ["dbg.log", "msgcount.log"]:
            with open(os.path.join(tmp, name), "rb") as f:
                files[name] = f.read()
        with open(os.path.join(tmp, "state.txt"), "rb") as f:
            files["state_sha.txt"], files["state_sel.txt"] = state_digest(f.read())
    os.makedirs(dest, exist_ok=True)
    for name, data in files.items():
        with gzip.GzipFile(os.path.join(dest, name + ".gz"), "wb", mtime=0) as g:
            g.write(data)
    return dest


def main_big():
    for c in BIG_CONFS:
        write_big_conf(c)
    with ThreadPoolExecutor(max_workers=6) as ex:
        for d in ex.map(lambda a: run_big(*a), BIG_RUNS):
            print("wrote", d, flush=True)


def main():
    if not os.path.exists(BIN):
        sys.exit("build the reference first: make -C oracle ref")
    if "--big" in sys.argv:
        main_big()
        return
    for conf in CONFS:
        for seed in SEEDS:
            for mode in MODES:
                run_one(conf, seed, mode, os.path.join(OUT, mode, conf, str(seed)))
    # the reference's own .conf inputs are data: keep copies beside the outputs
    os.makedirs(os.path.join(OUT, "testcases"), exist_ok=True)
    for conf in CONFS:
        shutil.copy(os.path.join(REF, "testcases", conf + ".conf"),
                    os.path.join(OUT, "testcases"))
    # the reference's committed golden log (singlefailure, node 5 failed; == seed 10 glibc)
    shutil.copy(os.path.join(REF, "dbg.log"), os.path.join(OUT, "reference_committed_dbg.log"))
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
