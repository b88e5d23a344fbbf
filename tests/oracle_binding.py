"""ctypes binding of oracle/liboracle.so -- the CPU checker (tests only).

The oracle is test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg load it, and only to CHECK or time-as-baseline the product.
"""
import ctypes
import gzip
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
GOLDEN = os.path.join(ROOT, "tests", "golden", "ref")
CONFS = ["singlefailure", "multifailure", "msgdropsinglefailure"]
SEEDS = [1, 5, 9, 10, 1234567]
MODES = ["glibc", "philox"]
FILES = ["dbg.log", "msgcount.log", "state.txt", "stdout.txt"]


MAX_FAIL_EVENTS = 8


class FailEvent(ctypes.Structure):
    _fields_ = [("tick", ctypes.c_int32), ("mode", ctypes.c_int32), ("ppm", ctypes.c_int32)]


class Policy(ctypes.Structure):
    """gsp_oracle_policy (oracle/gsp_oracle.h) == gsp_policy (include/gossip/gossip.h)."""
    _fields_ = [("drop_from", ctypes.c_int32), ("drop_until", ctypes.c_int32),
                ("step_rate", ctypes.c_double), ("intro_list", ctypes.c_int32),
                ("n_fail_events", ctypes.c_int32), ("fail_events", FailEvent * MAX_FAIL_EVENTS)]


def make_policy(drop_window=None, step_rate=0.0, intro_list=0, fail_events=()):
    """drop_window=(from, until); fail_events=[(tick, mode, ppm), ...]."""
    p = Policy()
    if drop_window:
        p.drop_from, p.drop_until = drop_window
    p.step_rate = step_rate
    p.intro_list = intro_list
    p.n_fail_events = len(fail_events)
    for i, (tk, md, pp) in enumerate(fail_events):
        p.fail_events[i] = FailEvent(tk, md, pp)
    return p


class ScaleCfg(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("fanout", ctypes.c_int32), ("drop_pct", ctypes.c_int32),
                ("tremove", ctypes.c_int32), ("h0", ctypes.c_int32), ("fail_mode", ctypes.c_int32),
                ("fail_tick", ctypes.c_int32), ("fail_ppm", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("tfail", ctypes.c_int32), ("swim", ctypes.c_int32),
                ("pol", Policy)]


class TickDigest(ctypes.Structure):
    _fields_ = [("tick", ctypes.c_int64), ("node_rounds", ctypes.c_int64),
                ("merges", ctypes.c_int64), ("sent", ctypes.c_int64),
                ("dropped", ctypes.c_int64), ("delivered", ctypes.c_int64),
                ("joins", ctypes.c_int64), ("removes", ctypes.c_int64),
                ("event_hash", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class PviewCfg(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("view", ctypes.c_int32), ("fanout", ctypes.c_int32),
                ("inbox", ctypes.c_int32), ("drop_pct", ctypes.c_int32),
                ("tremove", ctypes.c_int32), ("h0", ctypes.c_int32), ("fail_mode", ctypes.c_int32),
                ("fail_tick", ctypes.c_int32), ("fail_ppm", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("tfail", ctypes.c_int32), ("swim", ctypes.c_int32),
                ("pol", Policy), ("evict_order", ctypes.c_int32)]


class PviewDigest(ctypes.Structure):
    _fields_ = [("tick", ctypes.c_int64), ("node_rounds", ctypes.c_int64),
                ("merges", ctypes.c_int64), ("sent", ctypes.c_int64),
                ("dropped", ctypes.c_int64), ("delivered", ctypes.c_int64),
                ("overflow", ctypes.c_int64), ("joins", ctypes.c_int64),
                ("removes", ctypes.c_int64), ("evicts", ctypes.c_int64),
                ("event_hash", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_oracle = None


def load_oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"],
                           check=True, capture_output=True)
        L = ctypes.CDLL(ORACLE_SO)
        L.gsp_oracle_mp1_run.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int,
                                         ctypes.c_int] + [ctypes.c_char_p] * 4
        L.gsp_oracle_mp1_run.restype = ctypes.c_int
        L.gsp_oracle_mp1_buffer_full_rejects.restype = ctypes.c_int64
        L.gsp_oracle_mp1_set_intro_list.argtypes = [ctypes.c_int]
        L.gsp_oracle_mp1_merges.restype = ctypes.c_int64
        L.gsp_glibc_stream.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_int32),
                                       ctypes.c_int64]
        L.gsp_scale_oracle_create.argtypes = [ctypes.POINTER(ScaleCfg)]
        L.gsp_scale_oracle_create.restype = ctypes.c_void_p
        L.gsp_scale_oracle_destroy.argtypes = [ctypes.c_void_p]
        L.gsp_scale_oracle_step.argtypes = [ctypes.c_void_p, ctypes.POINTER(TickDigest)]
        L.gsp_scale_oracle_row.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.gsp_scale_oracle_own_hb.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.gsp_scale_oracle_fail_tick.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.gsp_scale_oracle_fail_tick.restype = ctypes.c_int32
        for pre in ("gsp_scale_oracle", "gsp_pview_oracle"):
            f = getattr(L, pre + "_start_tick")
            f.argtypes = [ctypes.c_void_p, ctypes.c_int32]
            f.restype = ctypes.c_int32
            f = getattr(L, pre + "_joinreps")
            f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
            f.restype = ctypes.c_int64
            f = getattr(L, pre + "_events")
            f.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 3 + [ctypes.c_int64]
            f.restype = ctypes.c_int64
        L.gsp_scale_oracle_messages.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int64]
        L.gsp_scale_oracle_messages.restype = ctypes.c_int64
        L.gsp_oracle_set_threads.argtypes = [ctypes.c_int]
        L.gsp_event_mix.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
        L.gsp_event_mix.restype = ctypes.c_uint64
        L.gsp_pview_oracle_create.argtypes = [ctypes.POINTER(PviewCfg)]
        L.gsp_pview_oracle_create.restype = ctypes.c_void_p
        L.gsp_pview_oracle_destroy.argtypes = [ctypes.c_void_p]
        L.gsp_pview_oracle_step.argtypes = [ctypes.c_void_p, ctypes.POINTER(PviewDigest)]
        L.gsp_pview_oracle_row.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.gsp_pview_oracle_row.restype = ctypes.c_int32
        L.gsp_pview_oracle_own_hb.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.gsp_pview_oracle_fail_tick.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.gsp_pview_oracle_fail_tick.restype = ctypes.c_int32
        L.gsp_pview_oracle_messages.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int64]
        L.gsp_pview_oracle_messages.restype = ctypes.c_int64
        L.gsp_pview_oracle_row_step.argtypes = [ctypes.POINTER(PviewCfg), ctypes.c_int32,
                                                ctypes.c_int32] + [ctypes.c_void_p] * 3 + [
            ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 8 + [ctypes.POINTER(PviewDigest)]
        L.gsp_pview_oracle_row_step.restype = ctypes.c_int32
        L.gsp_oracle_draw.argtypes = [ctypes.c_uint32, ctypes.c_uint64] + [ctypes.c_uint32] * 4
        L.gsp_oracle_draw.restype = ctypes.c_uint32
        _oracle = L
    return _oracle


def golden(mode, conf, seed, name):
    with gzip.open(os.path.join(GOLDEN, mode, conf, str(seed), name + ".gz"), "rb") as f:
        return f.read()


def conf_path(conf):
    if conf in BIG_CONFS:
        return os.path.join(GOLDEN_BIG, "testcases", conf + ".conf")
    return os.path.join(GOLDEN, "testcases", conf + ".conf")


# Fixtures past the reference's N = 10 (tests/golden/make_golden.py --big): MAX_NNB 70 / 300 /
# 600, made by the reference itself; state.txt is kept as per-tick SHA-256 + selected ticks.
GOLDEN_BIG = os.path.join(ROOT, "tests", "golden", "ref_big")
BIG_CONFS = ["n70_single", "n70_multi", "n70_drop", "n300_single", "n300_multi", "n300_drop",
             "n600_multidrop", "n600_single"]
BIG_RUNS = [(c, s, m) for c in BIG_CONFS if not c.startswith("n600") for s in (3, 77)
            for m in MODES] + [(c, 3, m) for c in BIG_CONFS if c.startswith("n600") for m in MODES]
BIG_FILES = ["dbg.log", "msgcount.log", "stdout.txt", "state_sha.txt", "state_sel.txt"]
STATE_SEL = (99, 100, 101, 121, 299, 300, 699)


def golden_big(mode, conf, seed, name):
    with gzip.open(os.path.join(GOLDEN_BIG, mode, conf, str(seed), name + ".gz"), "rb") as f:
        return f.read()


def state_digest(state_bytes):
    """(per-tick SHA-256 lines, lines of the STATE_SEL ticks) of a state dump -- the form the
    big fixtures keep (same function as tests/golden/make_golden.py)."""
    import hashlib
    by_tick = {}
    for line in state_bytes.splitlines(keepends=True):
        by_tick.setdefault(int(line.split(b" ", 1)[0]), []).append(line)
    sha = b"".join(b"%d %s\n" % (t, hashlib.sha256(b"".join(v)).hexdigest().encode())
                   for t, v in sorted(by_tick.items()))
    sel = b"".join(b"".join(by_tick.get(t, [])) for t in STATE_SEL)
    return sha, sel


def outputs_for_big(paths):
    """The BIG_FILES view of a run's output files (dbg / msgcount / stdout / state)."""
    out = {}
    for name in ["dbg.log", "msgcount.log", "stdout.txt"]:
        with open(paths[name], "rb") as f:
            out[name] = f.read()
    with open(paths["state.txt"], "rb") as f:
        out["state_sha.txt"], out["state_sel.txt"] = state_digest(f.read())
    return out


def run_oracle_mp1(conf, seed, mode, out_dir, ticks=700, intro_list=0):
    """intro_list: the exact engine's opt-in bounded introducer list (0 = the reference)."""
    L = load_oracle()
    os.makedirs(out_dir, exist_ok=True)
    p = lambda x: os.path.join(out_dir, x).encode()
    L.gsp_oracle_mp1_set_intro_list(intro_list)
    try:
        rc = L.gsp_oracle_mp1_run(conf_path(conf).encode(), seed, MODES.index(mode), ticks,
                                  p("dbg.log"), p("msgcount.log"), p("state.txt"),
                                  p("stdout.txt"))
    finally:
        L.gsp_oracle_mp1_set_intro_list(0)
    assert rc == 0, rc
    return {f: os.path.join(out_dir, f) for f in FILES}


class ScaleOracle:
    """The scale-protocol restatement (oracle/scale_oracle.c)."""
    _pre = "gsp_scale_oracle"

    def start_tick(self, r):
        return getattr(self.L, self._pre + "_start_tick")(self.h, r)

    def joinreps(self):
        import numpy as np
        f = getattr(self.L, self._pre + "_joinreps")
        n = f(self.h, None, 0)
        out = np.zeros(max(n, 1), np.int32)
        f(self.h, out.ctypes.data, n)
        return out[:n]

    def events(self):
        """(kind, r, x) arrays of the last step's events."""
        import numpy as np
        f = getattr(self.L, self._pre + "_events")
        n = f(self.h, None, None, None, 0)
        k, r, x = (np.zeros(max(n, 1), np.int32) for _ in range(3))
        f(self.h, k.ctypes.data, r.ctypes.data, x.ctypes.data, n)
        return k[:n], r[:n], x[:n]

    def __init__(self, n, fanout=3, drop_pct=0, tremove=20, h0=1, fail_mode=0, fail_tick=10,
                 fail_ppm=0, seed=0x5EED, tfail=0, swim=0, policy=None):
        self.L = load_oracle()
        self.cfg = ScaleCfg(n, fanout, drop_pct, tremove, h0, fail_mode, fail_tick, fail_ppm, seed,
                            tfail, swim, policy or Policy())
        self.h = self.L.gsp_scale_oracle_create(ctypes.byref(self.cfg))
        assert self.h, "oracle create failed"
        self.n = n

    def step(self):
        d = TickDigest()
        assert self.L.gsp_scale_oracle_step(self.h, ctypes.byref(d)) == 0
        return d.as_dict()

    def row(self, r):
        import numpy as np
        pres = np.zeros(self.n, np.uint8)
        hb = np.zeros(self.n, np.int32)
        ts = np.zeros(self.n, np.int32)
        self.L.gsp_scale_oracle_row(self.h, r, pres.ctypes.data, hb.ctypes.data, ts.ctypes.data)
        return pres, hb, ts

    def own_hb(self, r):
        return self.L.gsp_scale_oracle_own_hb(self.h, r)

    def fail_tick(self, r):
        return self.L.gsp_scale_oracle_fail_tick(self.h, r)

    def messages(self):
        import numpy as np
        n = self.L.gsp_scale_oracle_messages(self.h, None, None, 0)
        src = np.zeros(max(n, 1), np.int32)
        dst = np.zeros(max(n, 1), np.int32)
        self.L.gsp_scale_oracle_messages(self.h, src.ctypes.data, dst.ctypes.data, n)
        return src[:n], dst[:n]

    def close(self):
        if self.h:
            self.L.gsp_scale_oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def pview_row_step(cfg, t, r, own, senders, views):
    """oracle/pview_oracle.c's per-row rule for one row (gsp_pview_oracle_row_step).
    own / views[j]: (ids, hb, ts) with ascending ids and absolute ts; senders[j] sent views[j].
    Returns ((ids, hb, ts) of r's new view, the row's digest counts)."""
    import numpy as np
    L = load_oracle()
    V = cfg.view
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)
    oi, oh, ot = (i32(x) for x in own)
    k = len(senders)
    sid = np.zeros((max(k, 1), V), np.int32)
    shb = np.zeros_like(sid)
    sts = np.zeros_like(sid)
    slen = np.zeros(max(k, 1), np.int32)
    for j, (vi, vh, vt) in enumerate(views):
        m = len(vi)
        sid[j, :m], shb[j, :m], sts[j, :m], slen[j] = vi, vh, vt, m
    snd = i32(list(senders) or [0])
    out = [np.zeros(V, np.int32) for _ in range(3)]
    d = PviewDigest()
    m = L.gsp_pview_oracle_row_step(ctypes.byref(cfg), t, r, oi.ctypes.data, oh.ctypes.data,
                                    ot.ctypes.data, len(oi), k, snd.ctypes.data, sid.ctypes.data,
                                    shb.ctypes.data, sts.ctypes.data, slen.ctypes.data,
                                    out[0].ctypes.data, out[1].ctypes.data, out[2].ctypes.data,
                                    ctypes.byref(d))
    assert m >= 0
    return tuple(x[:m] for x in out), d.as_dict()


class PviewOracle:
    """The partial-view restatement (oracle/pview_oracle.c)."""
    _pre = "gsp_pview_oracle"

    def start_tick(self, r):
        return getattr(self.L, self._pre + "_start_tick")(self.h, r)

    def joinreps(self):
        import numpy as np
        f = getattr(self.L, self._pre + "_joinreps")
        n = f(self.h, None, 0)
        out = np.zeros(max(n, 1), np.int32)
        f(self.h, out.ctypes.data, n)
        return out[:n]

    def events(self):
        """(kind, r, x) arrays of the last step's events."""
        import numpy as np
        f = getattr(self.L, self._pre + "_events")
        n = f(self.h, None, None, None, 0)
        k, r, x = (np.zeros(max(n, 1), np.int32) for _ in range(3))
        f(self.h, k.ctypes.data, r.ctypes.data, x.ctypes.data, n)
        return k[:n], r[:n], x[:n]

    def __init__(self, n, view=256, fanout=3, inbox=7, drop_pct=0, tremove=20, h0=1,
                 fail_mode=0, fail_tick=10, fail_ppm=0, seed=0x5EED, tfail=0, swim=0, policy=None,
                 evict_order=0):
        self.L = load_oracle()
        self.cfg = PviewCfg(n, view, fanout, inbox, drop_pct, tremove, h0, fail_mode, fail_tick,
                            fail_ppm, seed, tfail, swim, policy or Policy(), evict_order)
        self.h = self.L.gsp_pview_oracle_create(ctypes.byref(self.cfg))
        assert self.h, "pview oracle create failed"
        self.n, self.view = n, view

    def step(self):
        d = PviewDigest()
        assert self.L.gsp_pview_oracle_step(self.h, ctypes.byref(d)) == 0
        return d.as_dict()

    def row(self, r):
        import numpy as np
        ids = np.zeros(self.view, np.int32)
        hb = np.zeros(self.view, np.int32)
        ts = np.zeros(self.view, np.int32)
        m = self.L.gsp_pview_oracle_row(self.h, r, ids.ctypes.data, hb.ctypes.data, ts.ctypes.data)
        return ids[:m], hb[:m], ts[:m]

    def own_hb(self, r):
        return self.L.gsp_pview_oracle_own_hb(self.h, r)

    def fail_tick(self, r):
        return self.L.gsp_pview_oracle_fail_tick(self.h, r)

    def messages(self):
        import numpy as np
        n = self.L.gsp_pview_oracle_messages(self.h, None, None, 0)
        src = np.zeros(max(n, 1), np.int32)
        dst = np.zeros(max(n, 1), np.int32)
        self.L.gsp_pview_oracle_messages(self.h, src.ctypes.data, dst.ctypes.data, n)
        return src[:n], dst[:n]

    def close(self):
        if self.h:
            self.L.gsp_pview_oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()
