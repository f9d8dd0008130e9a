"""In-process A/B helpers over the conv route table (csrc/kernels/conv_route.hip) for the
dev/tools harnesses: they replace the per-call TDL_GLDS_CFG_* environment knobs of earlier rounds
(now rows of the table, validated by conv_route_set)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402

RF_STATS, RF_JOIN, RF_FP8 = 1, 2, 8


def glds_cfg(op, cfg, need=0):
    """Every LDS-DMA row of `op` ('fwd' / 'dgrad' / 'wgrad') whose need-mask contains `need` onto
    tile config `cfg` (rows that do not instantiate it keep theirs); cfg None: back to each row's
    default."""
    e = ext()
    for r in e.conv_route_table():
        if r["op"] != op or r["impl"] != "glds" or r["need"] & RF_FP8 or (r["need"] & need) != need:
            continue
        c = r["default_cfg"] if cfg is None else int(cfg)
        if e.conv_route_cfg_instantiated(1, {"fwd": 0, "dgrad": 1, "wgrad": 2}[op], c, r["need"]):
            e.conv_route_set(r["name"], cfg=c)
