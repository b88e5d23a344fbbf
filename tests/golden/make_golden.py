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
import os
import shutil
import subprocess
import sys
import tempfile

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


def main():
    if not os.path.exists(BIN):
        sys.exit("build the reference first: make -C oracle ref")
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
