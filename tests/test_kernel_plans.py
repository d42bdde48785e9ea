"""Host-side kernel planning of the production library (no GPU needed: the HIP library's planning
functions run on the host): which layers and batches take the weight-stationary conv (tile 40), the
small-batch wgrad plan and the automatic wgrad / dgrad overlap."""
import pytest

from alphago_amd import ops

S2 = 361


@pytest.fixture(scope="module", autouse=True)
def _lib():
    try:
        ops.load()
    except Exception as e:  # noqa: BLE001 - no HIP runtime / library in this environment
        pytest.skip("production library not loadable here: %s" % e)


def test_weight_stationary_shapes():
    # the trunk layers of both nets and the policy's 5x5 first layer; not the value net's first layer
    assert ops.conv_ws_supported(192, 192, 3) and ops.conv_ws_supported(192, 64, 5)
    assert ops.conv_ws_supported(160, 160, 3) and ops.conv_ws_supported(128, 128, 3)
    assert ops.conv_ws_supported(64, 64, 3)
    assert not ops.conv_ws_supported(160, 64, 5)


def test_weight_stationary_batch_limits(monkeypatch):
    assert ops.ws_applies(1 * S2, 192, 192, 3) and ops.ws_applies(32 * S2, 192, 192, 3)
    assert not ops.ws_applies(33 * S2, 192, 192, 3)
    # inside training steps it stops at B = 16 (the side-stream wgrad shares the GPU there)
    assert ops.ws_applies(16 * S2, 192, 192, 3, training=True)
    assert not ops.ws_applies(17 * S2, 192, 192, 3, training=True)
    assert ops.ws_applies(32 * S2, 160, 160, 3) and not ops.ws_applies(17 * S2, 160, 160, 3, training=True)
    monkeypatch.setenv("ALPHAGO_AMD_WS", "0")
    assert not ops.ws_applies(1 * S2, 192, 192, 3)


@pytest.mark.parametrize("B,small", [(1, False), (16, False), (17, True), (32, True), (64, True), (65, False),
                                     (2176, False)])
def test_small_batch_wgrad_plan(B, small):
    var, ns = ops.wgrad_config(B * S2, 192, 192, 3)
    assert (var == ops.WGRAD_SMALL) == small
    assert ns >= 1
    if small:
        taps, per_split, per_cu, threads = ops.wgrad_plan(192, 192, 3, 0, ops.WGRAD_SMALL)
        assert (taps, per_split, per_cu) == (3, 27, 2)
        assert ns * per_split <= 256 * per_cu  # one resident round
    # the first layer (48 real planes) and the value net's 160-wide layers keep their own plans
    assert ops.wgrad_config(B * S2, 192, 64, 5, cin_real=48)[0] == 0
    assert ops.wgrad_config(B * S2, 160, 160, 3)[0] == 0


def test_automatic_overlap_range():
    from alphago_amd.train.engine import OVERLAP_AUTO_MAX_PIXELS, OVERLAP_AUTO_MIN_PIXELS

    assert OVERLAP_AUTO_MIN_PIXELS == 17 * S2 and OVERLAP_AUTO_MAX_PIXELS == 256 * S2
