"""Split-R-hat/ESS at the BASELINE configs' sizes: device result vs the
oracle's f32 restatement of stats.rs vs an f64 evaluation (tests/_diag_cases.py).
Writes one JSON line per config to the file given as argv[1] (default stdout)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import general_mcmc_amd as gm  # noqa: E402
from tests import _diag_cases as dc, _oracle  # noqa: E402


def main():
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else sys.stdout
    which = sys.argv[2].split(",") if len(sys.argv) > 2 else ["cfg2", "cfg4", "cfg5"]
    gm._lib.require_gpu()
    ora = _oracle.load()
    for name in which:
        t = time.time()
        res = getattr(dc, name)(gm, ora)
        res["config"] = name
        res["seconds"] = round(time.time() - t, 1)
        res["oracle_threads"] = dc.threads()
        print(json.dumps(res), file=out, flush=True)
        print(name, "done", res["seconds"], "s", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
