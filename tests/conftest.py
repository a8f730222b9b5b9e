import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "protein-structure-tokenizer_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "reference: runs the reference's own code under the test shim "
                                       "(needs /root/reference; skipped elsewhere)")


def pytest_collection_modifyitems(config, items):
    import _refenv
    if not _refenv.available():
        skip = pytest.mark.skip(reason="/root/reference not present")
        for it in items:
            if "reference" in it.keywords:
                it.add_marker(skip)


GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="session")
def casp14_dir(tmp_path_factory):
    """The 31 CASP14 PDB files (tests/golden/casp14_pdbs.tar.gz) extracted to a temp dir."""
    import tarfile
    d = tmp_path_factory.mktemp("casp14")
    with tarfile.open(os.path.join(GOLDEN, "casp14_pdbs.tar.gz")) as tf:
        for m in tf.getmembers():
            if m.isfile() and m.name.startswith("casp14_pdbs/") and m.name.endswith(".pdb") and ".." not in m.name:
                tf.extract(m, d)
    return os.path.join(str(d), "casp14_pdbs")
