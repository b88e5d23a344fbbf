"""The drop-in `Application` binaries on the GPU.

oracle/_ref/Application_facade is the reference's OWN Application.cpp (/root/reference,
unmodified), compiled against the forwarding headers include/gossip/ref/ and linked with
libgossip_amd.so (oracle/Makefile; a test binary, never the product).  Its time() is pinned by
GSP_SEED exactly as oracle/_ref/Application's is (oracle/ref_time_pin.c), so its two
srand(time(NULL)) calls (Application.cpp:50, 96) seed the engine with the golden run's seed:
* stdout, dbg.log and msgcount.log equal the reference's byte for byte, 3 testcases x 5 seeds x
  {glibc, philox} (GSP_RNG=philox: the engine's Philox stream, as oracle/_ref/Application_replay);
* with the wall-clock seed, Grader.sh's checks (tests/grader.py) give 90/90.

gossip_protocol_amd/bin/Application is the build's own Application-shaped driver
(gossip_protocol_amd/app/app_main.cpp) on the same facade.

It is built only from the MP1Node / EmulNet / Params / Log facade (include/gossip/
mp1_facade.hpp) and is run exactly the way Grader.sh runs the reference
(`./Application testcases/<case>.conf` in a directory that holds testcases/, Grader.sh:32-34):
* with the seed pinned, dbg.log, msgcount.log and stdout equal the reference's, byte for byte;
* with the default time(NULL) seed, Grader.sh's checks (restated in tests/grader.py)
  give 30/30 per scenario, 90/90 in total.
"""
import os
import shutil
import subprocess

import pytest

from tests.oracle_binding import CONFS, MODES, SEEDS, conf_path, golden
from tests import grader

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "gossip_protocol_amd", "bin", "Application")
REF_APP = os.path.join(ROOT, "oracle", "_ref", "Application_facade")


def _run(tmp, conf, env_extra, app=APP):
    os.makedirs(os.path.join(tmp, "testcases"), exist_ok=True)
    shutil.copy(conf_path(conf), os.path.join(tmp, "testcases"))
    env = dict(os.environ, **env_extra)
    r = subprocess.run([app, "testcases/%s.conf" % conf], cwd=tmp, env=env, capture_output=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    return r.stdout


def _need_ref_app():
    if not os.path.exists(REF_APP):
        pytest.fail("oracle/_ref/Application_facade is missing: build it here with `make -C oracle` "
                    "(it needs /root/reference and gossip_protocol_amd/libgossip_amd.so)")


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("conf", CONFS)
def test_reference_application_on_facade(tmp_path, conf, seed, mode):
    """The reference's unmodified Application.cpp on the engine = the reference, byte for byte."""
    _need_ref_app()
    env = {"GSP_SEED": str(seed)}
    if mode == "philox":
        env["GSP_RNG"] = "philox"
    else:
        env["GSP_RNG"] = "glibc"
    out = _run(str(tmp_path), conf, env, app=REF_APP)
    assert out == golden(mode, conf, seed, "stdout.txt")
    for name in ["dbg.log", "msgcount.log"]:
        with open(os.path.join(str(tmp_path), name), "rb") as f:
            assert f.read() == golden(mode, conf, seed, name), name
    assert os.path.exists(os.path.join(str(tmp_path), "stats.log"))


def test_reference_application_on_facade_grader_90(tmp_path):
    """Grader.sh's scenarios with the wall-clock seed (no GSP_SEED: time() is libc's)."""
    _need_ref_app()
    total = 0
    env = {k: v for k, v in os.environ.items() if k not in ("GSP_SEED", "GSP_RNG")}
    for conf in CONFS:
        d = os.path.join(str(tmp_path), conf)
        os.makedirs(os.path.join(d, "testcases"))
        shutil.copy(conf_path(conf), os.path.join(d, "testcases"))
        r = subprocess.run([REF_APP, "testcases/%s.conf" % conf], cwd=d, env=env,
                           capture_output=True, timeout=120)
        assert r.returncode == 0, r.stderr.decode()
        with open(os.path.join(d, "dbg.log"), "rb") as f:
            total += grader.score(f.read(), conf)
    assert total == 90


@pytest.mark.parametrize("mode", ["glibc", "philox"])
@pytest.mark.parametrize("seed", [1, 10])
@pytest.mark.parametrize("conf", CONFS)
def test_application_bitexact(tmp_path, conf, seed, mode):
    out = _run(str(tmp_path), conf, {"GSP_SEED": str(seed), "GSP_RNG": mode})
    assert out == golden(mode, conf, seed, "stdout.txt")
    for name in ["dbg.log", "msgcount.log"]:
        with open(os.path.join(str(tmp_path), name), "rb") as f:
            assert f.read() == golden(mode, conf, seed, name), name
    assert os.path.exists(os.path.join(str(tmp_path), "stats.log"))


def test_grader_directory_90():
    """grader/ is the layout Grader.sh drives unmodified: for each scenario it runs
    `make clean; make; ./Application testcases/<x>.conf` in that directory
    (/root/reference/Grader.sh:32-34, 81-83, 144-146) and greps dbg.log; tests/grader.py
    restates the greps.  The same command sequence here must score 90/90."""
    gdir = os.path.join(ROOT, "grader")
    env = {k: v for k, v in os.environ.items() if k not in ("GSP_SEED", "GSP_RNG")}
    total = 0
    try:
        for conf in CONFS:
            r = subprocess.run(["bash", "-c", "make clean > /dev/null && make > /dev/null && "
                                "./Application testcases/%s.conf > /dev/null" % conf],
                               cwd=gdir, env=env, capture_output=True, timeout=300)
            assert r.returncode == 0, r.stderr.decode()
            with open(os.path.join(gdir, "dbg.log"), "rb") as f:
                total += grader.score(f.read(), conf)
    finally:
        subprocess.run(["make", "clean"], cwd=gdir, capture_output=True)
    assert total == 90


def test_application_grader_90(tmp_path):
    total = 0
    env = {k: v for k, v in os.environ.items() if k not in ("GSP_SEED", "GSP_RNG")}
    for conf in CONFS:
        d = os.path.join(str(tmp_path), conf)
        os.makedirs(d)
        os.makedirs(os.path.join(d, "testcases"))
        shutil.copy(conf_path(conf), os.path.join(d, "testcases"))
        r = subprocess.run([APP, "testcases/%s.conf" % conf], cwd=d, env=env, capture_output=True,
                           timeout=120)
        assert r.returncode == 0
        with open(os.path.join(d, "dbg.log"), "rb") as f:
            total += grader.score(f.read(), conf)
    assert total == 90
