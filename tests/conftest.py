"""pytest configuration: the `gpu` marker, repo on sys.path, libraries built if missing.

The engine library is imported before anything imports torch (shared ROCm sonames: the
first loaded runtime wins, see assistedmanipulation_amd/_lib.py)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def _ensure_built():
    lib = os.path.join(REPO, "assistedmanipulation_amd", "lib", "libmppi_amd.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "assistedmanipulation_amd", "csrc")])
    orc = os.path.join(REPO, "oracle", "build", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])


_ensure_built()
import assistedmanipulation_amd  # noqa: E402,F401  (load the engine's ROCm runtime first)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU test")
