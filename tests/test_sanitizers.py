"""Sanitizer builds (CPU only): the oracle under AddressSanitizer + UndefinedBehaviorSanitizer
(oracle/asan_driver.c via `make -C oracle asan-run`), and the product's host-side code that handles
untrusted caller bytes and heap offsets -- the C-ABI decoder's SPS peek (csrc/host_sps.h) and the N-API
heap (napi/heap.h) -- fuzzed by tests/native/host_fuzz.cc under the same sanitizers."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ['-O1', '-g', '-fno-omit-frame-pointer', '-fsanitize=address,undefined', '-fno-sanitize-recover=all']
ENV = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=1', UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1')

pytestmark = pytest.mark.skipif(shutil.which('gcc') is None or shutil.which('g++') is None, reason='needs gcc/g++')


def test_oracle_under_asan_ubsan():
    r = subprocess.run(['make', '-s', '-C', os.path.join(ROOT, 'oracle'), 'asan-run'], capture_output=True, text=True,
                       env=ENV, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert 'asan_driver: ok' in r.stdout


def test_host_boundary_code_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / 'host_fuzz')
    o = os.path.join(ROOT, 'oracle')
    objs = []
    for src in ('h264o_common.c', 'h264o_enc.c', 'h264o_dec.c'):  # h264o_write_sps builds the intact SPS inputs
        obj = str(tmp_path / (src + '.o'))
        subprocess.run(['gcc', '-std=c11', '-c', '-o', obj, os.path.join(o, src)] + SAN, check=True)
        objs.append(obj)
    subprocess.run(['g++', '-std=c++17', '-Wall', '-Wextra', '-o', exe, os.path.join(ROOT, 'tests', 'native', 'host_fuzz.cc')] + objs + SAN,
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert 'host_fuzz: ok' in r.stdout
