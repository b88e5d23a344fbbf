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


class ScaleCfg(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("fanout", ctypes.c_int32), ("drop_pct", ctypes.c_int32),
                ("tremove", ctypes.c_int32), ("h0", ctypes.c_int32), ("fail_mode", ctypes.c_int32),
                ("fail_tick", ctypes.c_int32), ("fail_ppm", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("tfail", ctypes.c_int32), ("swim", ctypes.c_int32)]


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
                ("seed", ctypes.c_uint64)]


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
        L.gsp_scale_oracle_messages.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int64]
        L.gsp_scale_oracle_messages.restype = ctypes.c_int64
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
        _oracle = L
    return _oracle


def golden(mode, conf, seed, name):
    with gzip.open(os.path.join(GOLDEN, mode, conf, str(seed), name + ".gz"), "rb") as f:
        return f.read()


def conf_path(conf):
    return os.path.join(GOLDEN, "testcases", conf + ".conf")


def run_oracle_mp1(conf, seed, mode, out_dir, ticks=700):
    L = load_oracle()
    os.makedirs(out_dir, exist_ok=True)
    p = lambda x: os.path.join(out_dir, x).encode()
    rc = L.gsp_oracle_mp1_run(conf_path(conf).encode(), seed, MODES.index(mode), ticks,
                              p("dbg.log"), p("msgcount.log"), p("state.txt"), p("stdout.txt"))
    assert rc == 0, rc
    return {f: os.path.join(out_dir, f) for f in FILES}


class ScaleOracle:
    """The scale-protocol restatement (oracle/scale_oracle.c)."""

    def __init__(self, n, fanout=3, drop_pct=0, tremove=20, h0=1, fail_mode=0, fail_tick=10,
                 fail_ppm=0, seed=0x5EED, tfail=0, swim=0):
        self.L = load_oracle()
        self.cfg = ScaleCfg(n, fanout, drop_pct, tremove, h0, fail_mode, fail_tick, fail_ppm, seed,
                            tfail, swim)
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


class PviewOracle:
    """The partial-view restatement (oracle/pview_oracle.c)."""

    def __init__(self, n, view=256, fanout=3, inbox=7, drop_pct=0, tremove=20, h0=1,
                 fail_mode=0, fail_tick=10, fail_ppm=0, seed=0x5EED):
        self.L = load_oracle()
        self.cfg = PviewCfg(n, view, fanout, inbox, drop_pct, tremove, h0, fail_mode, fail_tick,
                            fail_ppm, seed)
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
