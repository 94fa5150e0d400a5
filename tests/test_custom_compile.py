"""CustomTarget sources compile through the runtime compiler (hiprtc) into
the engine's kernels on a machine without a GPU (the build container): the
embedded device headers are complete and self-contained."""
import numpy as np
import pytest

from tests import custom_targets as ct


@pytest.fixture(scope="module")
def gmc():
    import general_mcmc_amd as gm
    gm._lib.load()
    return gm


@pytest.mark.parametrize("sampler,dtype", [("logp", np.float64), ("hmc", np.float32), ("mh", np.float64)])
def test_custom_source_compiles(gmc, sampler, dtype):
    gmc.CustomTarget(ct.ROSENBROCK, 8, [1.0, 100.0]).check(sampler, dtype)


def test_custom_source_error_has_log(gmc):
    with pytest.raises(gmc.GMError, match="undeclared identifier 'undefined_symbol'"):
        gmc.CustomTarget(ct.BROKEN, 4).check("hmc")
