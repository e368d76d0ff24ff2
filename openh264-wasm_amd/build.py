"""Build libh264mi.so for gfx950 in-tree (openh264-wasm_amd/lib/). Used by __graft_entry__.build()."""
import os, subprocess, sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, 'csrc', 'h264mi_kernels.hip')
OUT = os.path.join(HERE, 'lib', 'libh264mi.so')


def build(force=False, verbose=False):
    deps = [os.path.join(HERE, 'csrc', f) for f in os.listdir(os.path.join(HERE, 'csrc'))]
    deps.append(os.path.join(os.path.dirname(HERE), 'include', 'h264mi.h'))
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(d) for d in deps):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = ['hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-shared', '-Wno-unused-result',
           '-Wno-pass-failed', '-o', OUT + '.tmp', SRC]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError('hipcc failed for libh264mi')
    if verbose:
        sys.stderr.write(r.stderr)
    os.replace(OUT + '.tmp', OUT)
    return OUT


NAPI_SRC = os.path.join(HERE, 'napi', 'h264mi_napi.cc')
NAPI_OUT = os.path.join(HERE, 'lib', 'h264mi.node')
NODE_INCLUDE = '/usr/include/node'


def build_napi(force=False):
    """Build the N-API addon lib/h264mi.node (the reference glue's Module over libh264mi) with g++ against
    the system Node headers. Returns its path, or None when Node's headers are not installed."""
    if not os.path.exists(os.path.join(NODE_INCLUDE, 'node_api.h')):
        return None
    lib = build(force=False)
    deps = [NAPI_SRC, lib, os.path.join(os.path.dirname(HERE), 'include', 'h264mi.h')]
    if not force and os.path.exists(NAPI_OUT) and os.path.getmtime(NAPI_OUT) >= max(os.path.getmtime(d) for d in deps):
        return NAPI_OUT
    cmd = ['g++', '-O2', '-std=c++17', '-shared', '-fPIC', '-Wall', '-I' + NODE_INCLUDE, '-o', NAPI_OUT + '.tmp', NAPI_SRC,
           '-L' + os.path.dirname(lib), '-lh264mi', '-Wl,-rpath,$ORIGIN']
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError('g++ failed for the N-API addon')
    os.replace(NAPI_OUT + '.tmp', NAPI_OUT)
    return NAPI_OUT


if __name__ == '__main__':
    print(build(force='-f' in sys.argv, verbose=True))
    print(build_napi(force='-f' in sys.argv))
