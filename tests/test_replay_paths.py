"""Which delayed-null decision path a length takes (tests/replay.py bounds):
the mask table for 2^m >= 2^14, float64 decisions for the other even
lengths <= 2^17 on the direct / Bluestein paths (not the single-workgroup
2^m <= 8192 kernel, not the scattering-tail extension), fp32 otherwise --
the rule the device follows (csrc/pss_pipeline.hip: refine_null, pss_run's
dispatch)."""
from tests import replay


def _case(tail=False):
    ops = [("make_pulses", 1.0, "pulses"), ("disperse", 10, "disperse"), ("null", 0.1, "null")]
    if tail:
        ops.insert(2, ("scatter_tail", 1e-4, 1400, None))
    return dict(ops=ops)


def test_packed64_lengths():
    c = _case()
    assert replay.packed64(30720, c)            # C4's fold-mode length (direct path)
    assert replay.packed64(10006, c)            # Bluestein
    assert replay.packed64(8192, c)             # single-workgroup kernel: float64 since round 6
    assert replay.packed64(4096, c)
    assert replay.packed64(64, c)               # the smallest single-workgroup length
    assert not replay.packed64(16384, c)        # mask-table four-step
    assert replay.packed64(32, c)               # 2^m < 64: direct DFT, refined
    assert replay.packed64(16, c)
    assert not replay.packed64(10007, c)        # odd: shift_t only
    assert not replay.packed64((1 << 17) + 2, c)
    assert not replay.packed64(30720, _case(tail=True))


def test_packed_bounds_tightened():
    assert replay.AMBIG_MAX_FRAC["packed"] <= 2e-3
    assert replay.FLIP_MAX_FRAC["packed"] <= 1e-5
    assert replay.AMBIG_MAX_FRAC["table"] <= 2e-3
    # fp32-decided lengths: ~10x the measured band (3.05e-5) and no flips
    assert replay.AMBIG_MAX_FRAC["packed_f32"] <= 3e-4
    assert replay.FLIP_MAX_FRAC["packed_f32"] <= 1e-5
