"""Test configuration. `-m "not gpu"`: oracle vs committed golden fixtures, host logic, C-ABI
library load/exports, gloo world_size-2 sharding. `-m gpu`: parity of the HIP path (through the
C-ABI) against the oracle on the same seeded inputs."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP path)')


@pytest.fixture(scope='session')
def oracle():
    """The CPU oracle (TEST INFRASTRUCTURE), built from oracle/ if needed."""
    so = os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so')
    if not os.path.exists(so):
        subprocess.run(['make', '-s', '-C', os.path.join(ROOT, 'oracle')], check=True)
    from _oracle import Oracle
    return Oracle(so)


@pytest.fixture(scope='session')
def libpath():
    so = os.path.join(ROOT, 'openh264-wasm_amd', 'lib', 'libh264mi.so')
    if not os.path.exists(so):
        sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
        import build
        build.build()
    return so


@pytest.fixture(scope='session')
def gpu_lib(libpath):
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    torch.cuda.set_device(0)
    import h264mi
    return h264mi.lib()
