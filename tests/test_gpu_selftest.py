"""Device arithmetic shortcuts proven exhaustively on the GPU (every input of their range)."""
import pytest

from halogen import abi


@pytest.mark.gpu
def test_fast_reciprocal_is_correctly_rounded(gpu):
    """rcp_exact (hg_device.h; self-test kernel in hg_selftest.hip): v_rcp_f32 + one FMA Newton step == IEEE 1.0f/x for all 2^32 bit patterns
    whose exponent field is in [2, 252] (x and 1/x normal); the rest take the IEEE division."""
    with abi.Context(0) as ctx:
        bad, tested = ctx.selftest(abi.HG_SELFTEST_RCP)
    assert tested == 251 * 2 * 2**23  # exponents 2..252, both signs, every mantissa
    assert bad == 0
