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


if __name__ == '__main__':
    print(build(force='-f' in sys.argv, verbose=True))
