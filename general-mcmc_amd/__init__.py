"""general_mcmc_amd — MI355X-native many-chain HMC / NUTS / Metropolis-Hastings.

Drop-in for the hot path of SauersML/general-mcmc (HMC, batched HMC, NUTS,
MH via ChainRunner, split-R-hat/ESS): the same facades and conventions, with
every transition computed by hand-written gfx950 HIP kernels in libgmcmc.so
(include/gmcmc.h is the C ABI). There is no CPU fallback.
"""
from . import _lib, batch_vector
from ._lib import GMError
from .core import init, init_det, init_with_seed
from .distributions import (CustomTarget, DenseGaussian, DiffableGaussian2D, Gaussian2D,
                            IsotropicGaussian, Rosenbrock2D, RosenbrockND)
from .hmc import HMC
from .metropolis_hastings import MetropolisHastings
from .nuts import NUTS, MassMatrix, NUTSChain, NUTSMassMatrixConfig
from .stats import (BasicStats, ChainStats, MultiChainTracker, Progress, RunStats, basic_stats,
                    split_rhat_mean_ess)

__all__ = [
    "HMC", "NUTS", "NUTSChain", "MetropolisHastings", "RosenbrockND", "Rosenbrock2D",
    "IsotropicGaussian", "DiffableGaussian2D", "DenseGaussian", "Gaussian2D", "CustomTarget", "init",
    "init_det",
    "init_with_seed", "split_rhat_mean_ess", "basic_stats", "BasicStats", "RunStats", "GMError",
    "batch_vector", "MultiChainTracker", "ChainStats", "Progress", "NUTSMassMatrixConfig", "MassMatrix",
]
