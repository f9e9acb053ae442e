import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")

# The drop-in modules are imported the way the reference's own tests import
# theirs (`from kmer import ...` from inside the source directory).
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libpa.so)")
    config.addinivalue_line("markers", "slow: longer-running test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def _library_line() -> str:
    """The loaded libpa.so's source hash against this checkout's (build_native.source_hash)."""
    try:
        import build_native
        import pa_native
        have = build_native.library_hash(pa_native.lib().pa_version().decode())
        want = build_native.source_hash()
        return f"libpa.so src={have[:16]} checkout={want[:16]} " + ("(match)" if have == want else "(MISMATCH)")
    except Exception as e:  # the summary line must not fail the run
        return f"libpa.so not loaded: {e}"


def pytest_report_header(config):
    return _library_line()


def pytest_terminal_summary(terminalreporter):
    terminalreporter.write_line(_library_line())
