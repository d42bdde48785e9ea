"""Test-parametrisation helpers.

Kernel-lab cases (kernels measured and recorded dead or slower: Winograd, the wgrad variants 1-8, the
forward-tile lab codes, the fp8 lab tilings, the GPU ladder reader) carry the ``lab`` mark; the default
GPU suite skips them (tests/conftest.py) and ``ALPHAGO_AMD_LAB_TESTS=1`` runs them."""
import pytest

LAB = pytest.mark.lab


def lab_params(values, production):
    """``values`` for a parametrize list, those not in ``production`` marked ``lab``."""
    return [v if v in production else pytest.param(v, marks=LAB) for v in values]
