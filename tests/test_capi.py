"""The C-ABI boundary (CPU only: no compute calls that need a GPU).

* libgossip_amd.so loads and exports every function include/gossip/gossip.h declares;
* the ctypes stub (gossip_protocol_amd/_lib.py) covers every declared function;
* Params parsing follows Params::setparams (Params.cpp:19-43);
* the host-side replay draw is the oracle's Philox, and matches Random123's KATs;
* without a GPU the engine constructors fail loudly (no silent CPU fallback).
"""
import ctypes
import os
import re

import pytest

from gossip_protocol_amd import _lib
from tests.oracle_binding import GOLDEN, load_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for hdr in ["include/gossip/gossip.h"]:
        src = open(os.path.join(ROOT, hdr)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[a-z_A-Z][\w \*]*?\b(gsp_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["gsp_create", "gsp_tick_recv", "gsp_tick_process", "gsp_scale_create",
                 "gsp_scale_step", "gsp_params_from_conf", "gsp_replay_draw"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_ctypes_stub_covers_header():
    missing = [n for n in declared_functions() if n not in _lib.SIGNATURES]
    assert not missing, missing
    _lib.lib()  # every signature binds


def test_params_from_conf():
    L = _lib.lib()
    for conf, want in [("singlefailure", (10, 1, 0)), ("multifailure", (10, 0, 0)),
                       ("msgdropsinglefailure", (10, 1, 1))]:
        p = _lib.GspParams()
        rc = L.gsp_params_from_conf(os.path.join(GOLDEN, "testcases", conf + ".conf").encode(),
                                    ctypes.byref(p))
        assert rc == 0
        assert (p.max_nnb, p.single_failure, p.drop_msg) == want
        assert abs(p.msg_drop_prob - 0.1) < 1e-12
        assert p.step_rate == 0.25 and p.max_msg_size == 4000 and p.tremove == 20
    p = _lib.GspParams()
    assert L.gsp_params_from_conf(b"/nonexistent.conf", ctypes.byref(p)) == -2
    assert b"cannot open" in L.gsp_last_error()


def test_replay_draw_matches_oracle():
    L = _lib.lib()
    O = load_oracle()
    O.gsp_oracle_draw.restype = ctypes.c_uint32
    O.gsp_oracle_draw.argtypes = [ctypes.c_uint32, ctypes.c_uint64] + [ctypes.c_uint32] * 4
    for dom in [0x53454E44, 0x4641494C, 0x50454552]:
        for seed in [0, 1, 10, 0x5EED, 2**40 + 7]:
            for a in range(0, 700, 97):
                args = (dom, seed, a, 3, 7, 3)
                assert L.gsp_replay_draw(*args) == O.gsp_oracle_draw(*args)


def test_product_philox_known_answer():
    L = _lib.lib()
    c = (ctypes.c_uint32 * 4)(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344)
    k = (ctypes.c_uint32 * 2)(0xa4093822, 0x299f31d0)
    o = (ctypes.c_uint32 * 4)()
    assert L.gsp_philox4x32_10(c, k, o) == 0
    assert tuple(o) == (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)


def test_no_gpu_fails_loudly():
    L = _lib.lib()
    if L.gsp_device_count() > 0:
        pytest.skip("a GPU is visible")
    p = _lib.GspParams()
    L.gsp_params_default(ctypes.byref(p))
    h = ctypes.c_void_p()
    assert L.gsp_create(ctypes.byref(p), 0, 0, 1, None, ctypes.byref(h)) != 0
    sp = _lib.GspScaleParams(n=1024, fanout=3, tremove=20, h0=1, max_ticks=16)
    assert L.gsp_scale_create(ctypes.byref(sp), 0, ctypes.byref(h)) != 0


def test_scale_variant_params_validated_before_the_device():
    """tfail / swim ranges are checked by the C ABI before any HIP call (GSP_ERR_INVALID = -1),
    in-range values get past validation (and fail later, at the device, without a GPU)."""
    L = _lib.lib()
    h = ctypes.c_void_p()
    base = dict(n=1024, fanout=3, tremove=20, h0=1, max_ticks=16)
    for bad in (dict(swim=-1), dict(swim=9), dict(tfail=20), dict(tfail=-2)):
        sp = _lib.GspScaleParams(**base, **bad)
        assert L.gsp_scale_create(ctypes.byref(sp), 0, ctypes.byref(h)) == -1, bad
    if L.gsp_device_count() == 0:
        for ok in (dict(swim=8), dict(tfail=5, swim=1)):
            sp = _lib.GspScaleParams(**base, **ok)
            assert L.gsp_scale_create(ctypes.byref(sp), 0, ctypes.byref(h)) not in (0, -1), ok


def test_struct_layouts_match_the_header():
    """Every public struct the ctypes stub mirrors has the C ABI's size."""
    L = _lib.lib()
    for name, cls in [("gsp_params", _lib.GspParams), ("gsp_member_view", _lib.GspMemberView),
                      ("gsp_entry", _lib.GspEntry), ("gsp_queued_msg", _lib.GspQueuedMsg),
                      ("gsp_exact_stats", _lib.GspExactStats),
                      ("gsp_fail_event", _lib.GspFailEvent), ("gsp_policy", _lib.GspPolicy),
                      ("gsp_scale_params", _lib.GspScaleParams),
                      ("gsp_scale_digest", _lib.GspScaleDigest),
                      ("gsp_scale_perf", _lib.GspScalePerf),
                      ("gsp_pview_params", _lib.GspPviewParams),
                      ("gsp_pview_digest", _lib.GspPviewDigest)]:
        assert L.gsp_struct_size(name.encode()) == ctypes.sizeof(cls), name
    assert L.gsp_abi_version() == 7


def test_scale_params_from_reference_conf():
    """The reference's own testcases parse unchanged (Params.cpp:22-25's four keys) into the
    scale protocol the way its driver uses them (Application.cpp:143, 177-200)."""
    from gossip_protocol_amd.scale import FAIL_HALF, FAIL_SINGLE, params_from_conf
    for conf, mode, drop in [("singlefailure", FAIL_SINGLE, 0), ("multifailure", FAIL_HALF, 0),
                             ("msgdropsinglefailure", FAIL_SINGLE, 10)]:
        p = params_from_conf(os.path.join(GOLDEN, "testcases", conf + ".conf"))
        assert (p.n, p.fail_mode, p.fail_tick, p.drop_pct) == (10, mode, 100, drop)
        assert p.policy.step_rate == 0.25 and p.max_ticks == 700 and p.tremove == 20
        # fail() sets dropmsg at the end of t = 50 and clears it at the end of t = 300: the
        # sends of ticks 51..300 are dropped (test_exact_gpu.py checks the exact driver agrees)
        assert (p.policy.drop_from, p.policy.drop_until) == ((51, 301) if drop else (0, 0))
        assert p.policy.intro_list == 0 and p.policy.n_fail_events == 0


def test_scale_params_extended_keys(tmp_path):
    from gossip_protocol_amd.pview import params_from_conf as pv_conf
    from gossip_protocol_amd.scale import FAIL_BLOCK, FAIL_RANDOM, params_from_conf
    path = str(tmp_path / "x.conf")
    with open(path, "w") as f:
        f.write("MAX_NNB: 10\nSINGLE_FAILURE: 1\nDROP_MSG: 1\nMSG_DROP_PROB: 0.2\n"
                "SCALE_N: 4096\nFANOUT: 5\nSEED: 77\nTICKS: 64\nSTEP_RATE: 0.01\n"
                "INTRO_LIST: 8\nDROP_WINDOW: 3 30\nFAIL: 20 RANDOM 10000\nFAIL: 25 BLOCK 50000\n"
                "FAIL: 40 3 0\nTFAIL: 5\nSWIM: 2\nEVENTS: 1\n\n")
    p = params_from_conf(path)
    assert (p.n, p.fanout, p.seed, p.max_ticks, p.drop_pct) == (4096, 5, 77, 64, 20)
    assert (p.fail_tick, p.fail_mode, p.fail_ppm) == (20, FAIL_RANDOM, 10000)
    assert p.policy.n_fail_events == 2
    assert (p.policy.fail_events[0].tick, p.policy.fail_events[0].mode) == (25, FAIL_BLOCK)
    assert (p.policy.drop_from, p.policy.drop_until, p.policy.intro_list) == (3, 30, 8)
    assert abs(p.policy.step_rate - 0.01) < 1e-12 and (p.tfail, p.swim, p.events) == (5, 2, 1)
    with open(path, "a") as f:
        f.write("VIEW: 64\nINBOX: 5\nEVICT_ORDER: 1\n")
    q = pv_conf(path)
    assert (q.n, q.view, q.inbox, q.fanout, q.tfail, q.swim) == (4096, 64, 5, 5, 5, 2)
    assert q.evict_order == 1
    L = _lib.lib()
    assert L.gsp_scale_params_from_conf(path.encode(), ctypes.byref(_lib.GspScaleParams())) == -1
    assert b"partial-view" in L.gsp_last_error()
    with open(path, "a") as f:
        f.write("BOGUS: 1\n")
    assert L.gsp_pview_params_from_conf(path.encode(), ctypes.byref(_lib.GspPviewParams())) == -1
    assert b"unknown key BOGUS" in L.gsp_last_error()


def test_fail_schedule_matches_oracle():
    """gsp_fail_schedule (host only) = the oracle's crash ticks, every mode and multi-event
    policies (the schedule bench.py uses to score failure detection from the event stream)."""
    import numpy as np
    from gossip_protocol_amd import _lib
    from gossip_protocol_amd.scale import make_policy
    from tests.oracle_binding import ScaleOracle
    from tests.oracle_binding import make_policy as oracle_policy
    ev = [(7, 3, 0), (9, 2, 40000)]
    for mode, ppm in ((1, 20000), (2, 50000), (3, 0), (4, 0)):
        for events in ((), ev):
            got = _lib.fail_schedule(3000, 77, mode, 5, ppm, make_policy(fail_events=list(events)))
            orc = ScaleOracle(3000, fail_mode=mode, fail_tick=5, fail_ppm=ppm,
                              seed=77, policy=oracle_policy(fail_events=list(events)))
            want = np.array([orc.fail_tick(r) for r in range(3000)], np.int32)
            orc.close()
            assert np.array_equal(got, want), (mode, events)
            assert (got < np.iinfo(np.int32).max).any()
