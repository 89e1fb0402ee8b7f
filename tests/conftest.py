"""Test configuration.

Markers: `gpu` = needs an MI355X (run with `-m gpu`); everything else runs on CPU only.
CPU tests exercise the oracle (test infrastructure, oracle/), the host code of the package and
the C-ABI library's symbol table; GPU tests call the product path through the C-ABI only.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'assistive-vr-gym_amd')
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP device); run with -m gpu')


@pytest.fixture(scope='session')
def scene():
    from avr import _abi as ABI
    A = ABI.load_scene()
    return A, ABI.ModelDesc(A)


@pytest.fixture(scope='session')
def oracle_built():
    from oracle import oracle
    oracle.build()
    return True


@pytest.fixture(scope='session')
def libavr_path():
    """The in-tree libavr.so; built here if missing (hipcc cross-compiles without a GPU)."""
    from avr import build
    return build.build_lib()
