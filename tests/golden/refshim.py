"""Import-time shim that lets the reference (/root/reference, pure PyTorch) be imported in
the build container to *generate* golden fixtures.  Test infrastructure only: nothing
under liteasr_amd/ imports this, and /root/reference never travels to the GPU box.

hydra / omegaconf / soundfile are not installed here; the reference only needs a few
names from them at import time, which are stood in below.  The
stand-ins are never on any arithmetic path.
"""

import sys
import types

REF = "/root/reference"


def install():
    if "liteasr" in sys.modules and getattr(sys.modules["liteasr"], "_shim", False):
        return sys.modules["liteasr"]
    om = types.ModuleType("omegaconf")
    om.II = lambda s: "${" + s + "}"
    om.MISSING = "???"

    class _OC:
        @staticmethod
        def merge(a, b):
            return b

        @staticmethod
        def set_struct(*a, **k):
            return None

    om.OmegaConf = _OC
    om.open_dict = None
    lc = types.ModuleType("omegaconf.listconfig")
    lc.ListConfig = list
    om.listconfig = lc
    sys.modules["omegaconf"] = om
    sys.modules["omegaconf.listconfig"] = lc

    hy = types.ModuleType("hydra")
    hc = types.ModuleType("hydra.core")
    cs = types.ModuleType("hydra.core.config_store")

    class _CS:
        @staticmethod
        def instance():
            return _CS()

        def store(self, *a, **k):
            return None

    cs.ConfigStore = _CS
    sys.modules["hydra"] = hy
    sys.modules["hydra.core"] = hc
    sys.modules["hydra.core.config_store"] = cs

    sf = types.ModuleType("soundfile")

    def _read(*a, **k):
        raise RuntimeError("soundfile stand-in: wav input is not used")

    sf.read = _read
    sys.modules["soundfile"] = sf

    pkg = types.ModuleType("liteasr")
    pkg.__path__ = [REF + "/liteasr"]
    pkg._shim = True
    sys.modules["liteasr"] = pkg
    return pkg
