"""The library's build record (gm_build_info, tools/source_digest.py): the
loaded libgmcmc.so carries the digest of the sources it was built from, it
equals this tree's, and a library whose digest differs is refused on load
with a rebuild message. CPU only: no device call."""
import pytest


def test_loaded_library_matches_tree():
    from general_mcmc_amd import _lib
    info = _lib.build_info(_lib.load())
    assert info["library"] is not None and info["library"].startswith("src:")
    assert info["tree"] == info["library"] and info["match"]


def test_stale_library_is_refused(monkeypatch):
    from general_mcmc_amd import _lib
    lib = _lib.load()
    real = _lib.build_info

    def stale(lib_=None):
        d = real(lib_)
        return dict(d, library="src:000000000000000000000000", match=False)

    monkeypatch.setattr(_lib, "build_info", stale)
    with pytest.raises(_lib.GMError, match="rebuild"):
        _lib._check_build(lib, "libgmcmc.so")


def test_digest_tool_covers_the_kernel_sources():
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("sd", os.path.join(root, "tools", "source_digest.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    files = [os.path.relpath(p, root) for p in mod.source_files()]
    for must in ("general-mcmc_amd/csrc/hmc_device.h", "general-mcmc_amd/csrc/nuts_device.h",
                 "general-mcmc_amd/csrc/mh_device.h", "general-mcmc_amd/csrc/gm_rng.h", "include/gmcmc.h",
                 "general-mcmc_amd/Makefile"):
        assert must in files
    assert len(mod.digest()) == 24
