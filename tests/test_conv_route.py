"""The conv route table on the CPU (no kernel runs): its rows are well-formed, every row's tile
config is one its kernel instantiates, overrides are validated, and the default routing of the
flagship ResNet-50 convs is pinned — a changed threshold shows up here as a diff, next to the
profile that justified the old one."""
import pytest

from tensorflowdistributedlearning_amd import _native

pytestmark = pytest.mark.skipif(not _native.available(), reason="native extension not built")

S, J, A, F8, W = 1, 2, 4, 8, 64
FWD, DGRAD, WGRAD = 0, 1, 2


@pytest.fixture()
def e():
    ext = _native.load()
    ext.conv_route_reset()
    ext.conv_set_glds_mode(-1)
    ext.conv_set_halo_mode(-1)
    ext.conv_set_pc(-1)
    yield ext
    ext.conv_route_reset()
    ext.conv_set_glds_mode(-1)
    ext.conv_set_halo_mode(-1)
    ext.conv_set_pc(-1)
    for op in (FWD, DGRAD, WGRAD):
        ext.conv_route_force(op, "")


def test_rows_are_well_formed(e):
    rows = e.conv_route_table()
    names = [r["name"] for r in rows]
    assert len(names) == len(set(names))
    for r in rows:
        assert r["instantiated"], r["name"]
        assert r["evidence"], r["name"]
        assert r["name"].startswith(r["op"] + "."), r["name"]
        assert r["taps"][0] <= r["taps"][1] and r["cin"][0] <= r["cin"][1]
        assert r["cout"][0] <= r["cout"][1]
        assert not (r["need"] & r["forbid"]), r["name"]
    # every op ends on the register-staged kernel, which takes anything the others refuse
    for op in ("fwd", "dgrad", "wgrad"):
        last = [r for r in rows if r["op"] == op][-1]
        assert last["impl"] == "gemm" and last["name"] == op + ".gemm"


# (H_out, Cin, Cout, k, stride) of ResNet-50 at batch 256; default rows for fwd (with BN
# statistics), dgrad (fused BN-backward sums; stride 1: flipped filter available), wgrad
RESNET50 = [
    ((56, 64, 64, 1, 1), "fwd.glds.1x1n64", "dgrad.asfwd.glds.n64", "wgrad.gemm"),
    ((56, 64, 64, 3, 1), "fwd.halo.rw64", "dgrad.asfwd.rw64", "wgrad.gemm"),
    ((56, 64, 256, 1, 1), "fwd.glds.wide", "dgrad.asfwd.glds.n64", "wgrad.glds.1x1"),
    ((56, 256, 64, 1, 1), "fwd.glds.1x1n64", "dgrad.asfwd.glds", "wgrad.gemm"),
    ((28, 128, 128, 3, 2), "fwd.glds.wide", "dgrad.glds.stats", "wgrad.gemm"),
    ((28, 128, 128, 3, 1), "fwd.glds.wide", "dgrad.asfwd.glds", "wgrad.halo.wide3x3"),
    ((14, 256, 256, 3, 1), "fwd.pc.wide3x3", "dgrad.asfwd.glds", "wgrad.halo.wide3x3"),
    ((14, 1024, 256, 1, 1), "fwd.glds.wide", "dgrad.asfwd.glds", "wgrad.glds.1x1"),
    ((7, 512, 512, 3, 1), "fwd.pc.wide3x3", "dgrad.asfwd.glds", "wgrad.gemm"),
    ((7, 1024, 2048, 1, 2), "fwd.glds.wide", "dgrad.glds.stats", "wgrad.glds.1x1"),
]


@pytest.mark.parametrize("shape,fwd,dgrad,wgrad", RESNET50)
def test_resnet50_default_routes(e, shape, fwd, dgrad, wgrad):
    H, ci, co, k, s = shape
    N = 256
    assert e.conv_route_select(FWD, k * k, s, ci, co, N * H * H, S)[0] == fwd
    Hin = H * s
    dflags = S | (W if s == 1 else 0)
    assert e.conv_route_select(DGRAD, k * k, s, ci, co, N * Hin * Hin, dflags)[0] == dgrad
    assert e.conv_route_select(WGRAD, k * k, s, ci, co, N * H * H, 0)[0] == wgrad


def test_dgrad_variants(e):
    rows = 256 * 56 * 56
    # no statistics: the producer/consumer dgrad-as-forward for wide 3x3s, the resident-filter
    # halo one for 64 -> 64 and the streaming halo one for other narrow ones
    assert e.conv_route_select(DGRAD, 9, 1, 256, 256, 256 * 14 * 14, W)[0] == "dgrad.asfwd.pc"
    assert e.conv_route_select(DGRAD, 9, 1, 64, 64, rows, W)[0] == "dgrad.asfwd.rw64"
    assert e.conv_route_select(DGRAD, 9, 1, 64, 128, rows, W)[0] == "dgrad.asfwd.halo"
    # statistics + join: the forward K loop's 256×128 tiles with a flipped filter (its 8-wave
    # tiles for narrow dx), else the DGRAD kernel's 8-wave ones
    f = S | J | 128 | W
    assert e.conv_route_select(DGRAD, 1, 1, 256, 1024, 256 * 14 * 14, f)[0] == \
        "dgrad.asfwd.glds.join.wide"
    assert e.conv_route_select(DGRAD, 1, 1, 64, 256, 256 * 56 * 56, f)[0] == "dgrad.asfwd.glds.join"
    assert e.conv_route_select(DGRAD, 1, 1, 256, 1024, 256 * 14 * 14, f & ~W)[0] == \
        "dgrad.glds.stats.join"
    # no flipped filter: the DGRAD kernel
    assert e.conv_route_select(DGRAD, 9, 1, 128, 128, 256 * 28 * 28, S)[0] == "dgrad.glds.stats"
    # strided with the per-class flipped sub-filters: one forward conv per parity class
    st = S | W | 256
    cls = [256 * 28 * 28] * 4
    assert e.conv_route_select(DGRAD, 9, 2, 128, 128, 256 * 56 * 56, st, cls)[0] == \
        "dgrad.asfwd.strided"
    assert e.conv_route_select(DGRAD, 9, 2, 64, 64, 256 * 56 * 56, st, cls)[0] == \
        "dgrad.asfwd.strided.n64"
    # ... not with statistics + join
    assert e.conv_route_select(DGRAD, 1, 2, 256, 512, 256 * 56 * 56, st | J | 128, cls[:1])[0] \
        == "dgrad.glds.stats.join"
    # fp8 rows ignore the LDS-DMA mode switch (no other kernel has fp8 operands)
    e.conv_set_glds_mode(0)
    assert e.conv_route_select(DGRAD, 9, 1, 64, 128, 4096, F8)[0] == "dgrad.glds.fp8.n64"
    assert e.conv_route_select(DGRAD, 9, 1, 128, 128, rows, S) == ["dgrad.gemm"]
    # fp8 with K % 128 != 0: no row (the launcher raises)
    assert e.conv_route_select(DGRAD, 9, 1, 128, 64, rows, F8) == []


def test_stem_forward_row(e):
    # the row-packed stem: 7 taps x 24 channels -> 64 at 112x112 (b256)
    assert e.conv_route_select(FWD, 7, 2, 24, 64, 256 * 112 * 112, S)[0] == "fwd.gemm"  # opt-in
    e.conv_route_set("fwd.glds.stem", on=1)
    assert e.conv_route_select(FWD, 7, 2, 24, 64, 256 * 112 * 112, S)[0] == "fwd.glds.stem"


def test_small_problems_stay_on_the_gemm(e):
    # < 128 tiles of 256x128: the register-staged kernel (DeepLab 13x13x1024->256 at b64)
    assert e.conv_route_select(FWD, 1, 1, 1024, 256, 64 * 13 * 13, 0)[0] == "fwd.gemm"
    # glds mode 2 (the kernel tests): size thresholds off, the test rows on
    e.conv_set_glds_mode(2)
    assert e.conv_route_select(FWD, 1, 1, 1024, 256, 64 * 13 * 13, 0)[0] == "fwd.glds.wide"
    assert e.conv_route_select(FWD, 9, 1, 64, 96, 500, 0)[0] == "fwd.glds.aligned"
    assert e.conv_route_select(FWD, 9, 1, 64, 40, 500, 0)[0] == "fwd.glds.aligned.n64"


def test_mode_switches(e):
    e.conv_set_halo_mode(0)
    assert e.conv_route_select(FWD, 9, 1, 64, 64, 256 * 56 * 56, S)[0] == "fwd.gemm"
    e.conv_set_halo_mode(2)
    assert e.conv_route_select(FWD, 9, 1, 64, 256, 500, S)[0] == "fwd.halo.aligned"
    e.conv_set_halo_mode(-1)
    e.conv_set_pc(0)  # the producer/consumer forward off: its rows drop out
    assert e.conv_route_select(FWD, 9, 1, 256, 256, 256 * 14 * 14, S)[0] == "fwd.glds.wide"


def test_overrides_are_validated(e):
    with pytest.raises(RuntimeError, match="unknown conv route"):
        e.conv_route_set("fwd.glds.nope", on=0)
    with pytest.raises(RuntimeError, match="not instantiated"):
        e.conv_route_set("fwd.glds.wide", cfg=7)  # the 64x256 config exists for WGRAD only
    with pytest.raises(RuntimeError, match="not instantiated"):
        e.conv_route_set("dgrad.glds.stats.aff", cfg=0)  # the folded-BN mask: cfg 4 / 6 only
    with pytest.raises(RuntimeError, match="not instantiated"):
        e.conv_route_set("fwd.halo.narrow", cfg=2)
    e.conv_route_set("dgrad.glds.stats", cfg=6)
    row = next(r for r in e.conv_route_table() if r["name"] == "dgrad.glds.stats")
    assert row["cfg"] == 6 and row["default_cfg"] == 0
    e.conv_route_set("fwd.glds.1x1n64", on=0)
    assert e.conv_route_select(FWD, 1, 1, 256, 64, 256 * 56 * 56, S)[0] == "fwd.gemm"
    e.conv_route_reset()
    assert e.conv_route_select(FWD, 1, 1, 256, 64, 256 * 56 * 56, S)[0] == "fwd.glds.1x1n64"
    # the opt-in stem weight gradient
    assert "wgrad.glds.stem" not in e.conv_route_select(WGRAD, 7, 1, 24, 64, 256 * 112 * 112, 0)
    e.conv_route_set("wgrad.glds.stem", on=1)
    assert e.conv_route_select(WGRAD, 7, 1, 24, 64, 256 * 112 * 112, 0)[0] == "wgrad.glds.stem"


def test_force(e):
    e.conv_route_force(FWD, "fwd.glds.aligned.n64")
    assert e.conv_route_select(FWD, 9, 1, 64, 64, 100, 0) == ["fwd.glds.aligned.n64"]
    assert e.conv_route_select(FWD, 9, 1, 64, 128, 100, 0) == []  # outside its window
    with pytest.raises(RuntimeError, match="no route"):
        e.conv_route_force(FWD, "dgrad.gemm")
    e.conv_route_force(FWD, "")
    assert e.conv_route_select(FWD, 9, 1, 64, 64, 100, 0)[0] == "fwd.gemm"
