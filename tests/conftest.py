import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "omero-ms-pixel-buffer_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def oracle():
    import _oracle
    _oracle.lib()
    return _oracle


@pytest.fixture(scope="session")
def service():
    import pbx
    s = pbx.PixelsService()
    yield s
    s.close()


@pytest.fixture(scope="session")
def staged_service():
    """Filter-None rows staged in a stream buffer by k_rows (the default reads the plane
    directly inside the deflate kernels)."""
    import pbx
    s = pbx.PixelsService(stage_rows=True)
    yield s
    s.close()


@pytest.fixture(scope="session", params=["direct", "staged"])
def png_service(request, service, staged_service):
    return service if request.param == "direct" else staged_service


@pytest.fixture(scope="session")
def adaptive_service():
    import pbx
    s = pbx.PixelsService(png_filter=pbx.FILTER_ADAPTIVE, tiff_deflate=True)
    yield s
    s.close()
