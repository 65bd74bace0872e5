"""Load the product package (its directory name is not a Python identifier)
and the test-only oracle."""
import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG_DIR = ROOT / "orb_slam2_modification_with-point-and-line-feature_amd"


def load_pkg():
    if "orbpl" in sys.modules:
        return sys.modules["orbpl"]
    spec = importlib.util.spec_from_file_location("orbpl", PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["orbpl"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    from oracle import oracle
    return oracle
