#!/usr/bin/env python3
"""Phase-stub and fixed-trip variants of the partial-view tick kernel ("Round 5:
SALU attribution").  Writes build/stub/<name>.hip from gossip_protocol_amd/csrc/pview_kernels.hip;
build each with `bash scripts/pv_variant.sh <name> build/stub/<name>.hip` and compare them with
`bash scripts/ab_pview_pmc.sh <tag> base <name>...` on a GPU box.

    nofold   every key its own entry: no run walk, no sender-event or orphan logic (wrong views)
    corank   no co-rank search (wrong merges)
    notree   keys left in block order (wrong merges)
    lift     co-rank by binary lifting: fixed trips, selects (same results)

Round 5 kept a fixed-trip run continuation in the product (it replaced a `while` over the
following keys: -1.8 % on the driver's window); the variants above patch the product as it is.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "gossip_protocol_amd", "csrc", "pview_kernels.hip")
OUT = os.path.join(HERE, "..", "build", "stub")

CORANK = """            int32_t lo = o > sb ? o - sb : 0, hi = o < sa ? o : sa;
            while (lo < hi) {                                  // co-rank of output o
                const int32_t mid = (lo + hi) >> 1;
                if (A[mid] < B[o - mid - 1]) lo = mid + 1; else hi = mid;
            }"""

LIFT = """            // co-rank of output o by binary lifting: the smallest i in [lo, hi] with
            // !(A[i] < B[o - i - 1]); fixed trips (log2 s + 1), selects instead of a loop
            int32_t lo = o > sb ? o - sb : 0;
            const int32_t hi = o < sa ? o : sa;
#pragma unroll
            for (int32_t step = s; step > 0; step >>= 1) {
                const int32_t c = lo + step;
                const bool in = c <= hi;
                const bool ok = in && A[in ? c - 1 : 0] < B[in ? o - c : 0];
                lo = ok ? c : lo;
            }"""

NO_CORANK = """            int32_t lo = o > sb ? o - sb : 0, hi = o < sa ? o : sa;
            lo = (lo + hi) >> 1;                               // STUB: no co-rank search"""

FOLD_HEAD = """#pragma unroll
    for (int e = 0; e < Q; ++e) {
        res[e] = 0;
        rid[e] = 0;
        const uint32_t key = ck[e];"""

NO_FOLD = """#pragma unroll
    for (int e = 0; e < Q; ++e) {                      // STUB: no run fold
        const uint32_t key = ck[e];
        const bool ok = key != kKeyMax && ((t5 - vv[e]) & 31u) < tr && vv[e] != 0u;
        res[e] = ok ? vv[e] : 0u;
        rid[e] = key_id(key);
        nloc += ok ? 1u : 0u;
    }
    (void)ax; (void)av; (void)ae0; (void)ajs; (void)aown; (void)adone; (void)hi_id; (void)next_key;
"""


def main():
    src = open(SRC).read()
    os.makedirs(OUT, exist_ok=True)
    assert CORANK in src and FOLD_HEAD in src, "pview_kernels.hip changed: update the patches"
    variants = {"lift": src.replace(CORANK, LIFT), "corank": src.replace(CORANK, NO_CORANK)}
    a = src.index("            const uint32_t *X = sh.kb(cur);")
    b = src.index("            if constexpr (!Sh::kInPlace) lds_store<Qt>(sh.kb(cur ^ 1) + begt, outk);")
    variants["notree"] = (src[:a] + "            const uint32_t *X = sh.kb(cur);\n#pragma unroll\n"
                          "            for (int e = 0; e < Qt; ++e) outk[e] = X[begt + e < P ? begt + e : P - 1];"
                          "   // STUB: no merge\n" + src[b:])
    f0 = src.index(FOLD_HEAD)
    f1 = src.index("    // orphans: senders in this lane's bracket that no list holds")
    variants["nofold"] = src[:f0] + NO_FOLD + src[f1:]
    for name in sys.argv[1:] or variants:
        path = os.path.join(OUT, name + ".hip")
        open(path, "w").write(variants[name])
        print(path)


if __name__ == "__main__":
    main()
