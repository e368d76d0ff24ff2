"""The N-API boundary: lib/h264mi.node + js/h264.js give the reference's JS glue the Emscripten
Module it binds (cwrap / _malloc / _free / getValue / bare HEAPU8), over libh264mi on the GPU.

CPU: the addon builds against the system Node headers, loads, and exports the wrapper surface.
GPU: tests/js/replay_workers.js replays the encoder_worker.js / decoder_worker.js call sequences
(one encoder Worker, decoder Workers under global stream indices, SharedArrayBuffer ring with
reference counts) and its outputs are checked byte for byte against the CPU oracle."""
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which('node')
pytestmark = pytest.mark.skipif(NODE is None or not os.path.exists('/usr/include/node/node_api.h'),
                                reason='Node.js / N-API headers not installed')
WRAPPER = ['init_encoder', 'force_key_frame', 'init_decoder', 'deinit_decoder', 'encode_frame', 'encode_frame_yuv_i420',
           'decode_frame_optimized', 'decode_frame_yuv_i420', 'free_buffer']


@pytest.fixture(scope='module')
def addon(libpath):
    sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
    import build
    return build.build_napi()


def test_addon_loads_and_exports(addon):
    r = subprocess.run([NODE, '-e', f"const m = require({json.dumps(addon)}); console.log(JSON.stringify(Object.keys(m)), m.version())"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    keys = json.loads(r.stdout.split(' h264mi')[0])
    for n in WRAPPER + ['createHeap', 'malloc', 'free']:
        assert n in keys, n
    assert 'h264mi' in r.stdout


def test_module_shim_syntax():
    for f in ('openh264-wasm_amd/js/h264.js', 'tests/js/replay_workers.js'):
        r = subprocess.run([NODE, '--check', os.path.join(ROOT, f)], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize('w,h,nf,streams,workers,mode', [(176, 144, 6, 3, 2, 'yuv'), (320, 240, 4, 2, 1, 'rgba')],
                         ids=['qcif-yuv-3streams', 'qvga-rgba'])
def test_worker_replay_bit_exact(addon, oracle, tmp_path, w, h, nf, streams, workers, mode):
    from h264mi.synth import SyntheticStream
    g = SyntheticStream(7, w, h)
    frames = [np.ascontiguousarray(g.frame(t)) for t in range(nf)]
    (tmp_path / 'in.yuv').write_bytes(b''.join(f.tobytes() for f in frames))
    out = tmp_path / 'out'
    r = subprocess.run([NODE, os.path.join(ROOT, 'tests', 'js', 'replay_workers.js'), str(tmp_path / 'in.yuv'), str(w), str(h),
                        str(nf), str(out), str(streams), str(workers), mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'replay ok' in r.stdout
    oe, od = oracle.encoder(w, h, 1000000), oracle.decoder()
    ref_units, ref_pics = [], []
    for f in frames:
        nal = oe.encode(f)
        ref_units.append(nal)
        if not nal:  # skipped by the rate control: the encoder worker posts 'skipped', nothing is decoded
            continue
        rc, pic, _, _ = od.decode(nal)
        assert rc == 1
        ref_pics.append(pic)
    assert json.loads((out / 'sizes.json').read_text()) == [len(u) for u in ref_units]
    assert (out / 'enc.h264').read_bytes() == b''.join(ref_units)
    for s in range(streams):
        got = (out / f'dec_{s}.{mode}').read_bytes()
        if mode == 'yuv':
            assert got == b''.join(p.tobytes() for p in ref_pics), f'stream {s}'
        else:
            assert got == b''.join(oracle.i420_to_rgba(p, w, h).tobytes() for p in ref_pics), f'stream {s}'
