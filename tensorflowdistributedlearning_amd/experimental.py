"""Experimental paths: built, tested for exactness, and measured SLOWER on MI355X than the defaults —
kept for A/B and as starting points, never on unless asked for.  One switch turns them on:

    TDL_EXPERIMENTAL=bnconv,join_stats,m32,stem_glds   (any subset; "all" for every one)

Each entry maps to the knob its code reads (set here, before any module reads it, when the package
is imported).  The measurement behind each verdict is in ``profiles/``.
"""
from __future__ import annotations

import os

# name: (what it is, the knob it sets, evidence)
FEATURES = {
    "bnconv": ("training BN + ReLU folded into the consuming dense conv (conv_pc.hip producer waves "
               "stage relu(a·z+b); ops/bnconv.py)", ("TDL_EXP_BNCONV", "1"),
               "profiles/r05_bnconv_fold_ab.txt: ResNet-50 b1024 11,676 vs 13,364 img/s"),
    "join_stats": ("residual-join BN-backward sums in the join's last dgrad (ops/gradjoin.py "
                   "TDL_BNSTAT_FUSE=1)", ("TDL_BNSTAT_FUSE", "1"),
                   "round 5: 12,990 / 12,992 vs 13,179 / 13,170 img/s (dev/scripts/gpu_r05_statsjoin.sh)"),
    "m32": ("32x32x16 MFMA blocks in the LDS-DMA forward / transposed-weight dgrad K loop "
            "(conv_glds.hip M32)", ("TDL_M32", "1"),
            "profiles/r03_m32_kloop_ab.txt: fwd -1.4 %, dgrad +1.7 %"),
    "stem_glds": ("row-packed ResNet stem on the LDS-DMA 8-wave tiles (route row fwd.glds.stem)",
                  ("TDL_ROUTE_ON", "fwd.glds.stem"),
                  "profiles/r05_stem_ab.txt: 914 vs 1017 us alone, no step gain"),
}


def requested():
    v = os.environ.get("TDL_EXPERIMENTAL", "")
    names = {n.strip() for n in v.replace(";", ",").split(",") if n.strip()}
    if "all" in names:
        names = set(FEATURES)
    unknown = names - set(FEATURES)
    if unknown:
        raise ValueError(f"TDL_EXPERIMENTAL: unknown feature(s) {sorted(unknown)}; "
                         f"known: {sorted(FEATURES)}")
    return names


def enabled(name: str) -> bool:
    return name in requested()


def apply_env():
    """Set the knobs of the requested features (an explicitly set knob wins)."""
    for name in requested():
        key, val = FEATURES[name][1]
        if key == "TDL_ROUTE_ON":
            cur = os.environ.get(key, "")
            if val not in cur.split(","):
                os.environ[key] = (cur + "," + val).strip(",")
        else:
            os.environ.setdefault(key, val)


apply_env()
