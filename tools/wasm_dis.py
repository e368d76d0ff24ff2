#!/usr/bin/env python3
"""Static disassembler for the reference's prebuilt scripts/h264.wasm (READ AS BYTES, NEVER EXECUTED).

Test infrastructure / study aid. It decodes the module's sections and every function body into a folded,
C-like listing so that OpenH264's encoder logic can be READ: which constants its parameter-set writers
put into the stream, which rules its rate control applies. Nothing is instantiated, interpreted,
translated into something runnable or linked; the listing is text for a human and for
`tools/wasm_tables.py`, which cites the file offsets it finds.

Listing conventions: `L3` = local 3 (parameters first), `G0` = global 0, `t17` = the result of a call,
`u8[x+4]` / `i32[x+12]` = loads (signed: `s8`, `s16`), stores are `i32[x+12] = v`; every statement carries
the file offset of the instruction that ends it (`@123456`).

  python tools/wasm_dis.py [--wasm PATH] [--out DIR] [--func N ...]
"""
import argparse
import os
import re
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from wasm_tables import DEFAULT_WASM, sections, sleb, uleb  # noqa: E402

VT = {0x7f: 'i32', 0x7e: 'i64', 0x7d: 'f32', 0x7c: 'f64', 0x7b: 'v128', 0x70: 'funcref', 0x6f: 'externref'}

LOADS = {0x28: ('i32', 'i32'), 0x29: ('i64', 'i64'), 0x2a: ('f32', 'f32'), 0x2b: ('f64', 'f64'),
         0x2c: ('s8', 'i32'), 0x2d: ('u8', 'i32'), 0x2e: ('s16', 'i32'), 0x2f: ('u16', 'i32'),
         0x30: ('s8', 'i64'), 0x31: ('u8', 'i64'), 0x32: ('s16', 'i64'), 0x33: ('u16', 'i64'),
         0x34: ('s32', 'i64'), 0x35: ('u32', 'i64')}
STORES = {0x36: 'i32', 0x37: 'i64', 0x38: 'f32', 0x39: 'f64', 0x3a: 'u8', 0x3b: 'u16', 0x3c: 'u8', 0x3d: 'u16',
          0x3e: 'u32'}

# numeric opcodes: (arity, operator or name)
UN = {0x45: 'i32.eqz', 0x50: 'i64.eqz', 0x67: 'clz', 0x68: 'ctz', 0x69: 'popcnt', 0x79: 'clz64', 0x7a: 'ctz64',
      0x7b: 'popcnt64', 0x8b: 'fabs', 0x8c: 'fneg', 0x8d: 'ceil', 0x8e: 'floor', 0x8f: 'trunc', 0x90: 'nearest',
      0x91: 'sqrt', 0x99: 'fabs', 0x9a: 'fneg', 0x9b: 'ceil', 0x9c: 'floor', 0x9d: 'trunc', 0x9e: 'nearest',
      0x9f: 'sqrt', 0xa7: 'i32.wrap', 0xa8: 'i32.trunc_f32_s', 0xa9: 'i32.trunc_f32_u', 0xaa: 'i32.trunc_f64_s',
      0xab: 'i32.trunc_f64_u', 0xac: 'i64.ext_s', 0xad: 'i64.ext_u', 0xae: 'i64.trunc_f32_s', 0xaf: 'i64.trunc_f32_u',
      0xb0: 'i64.trunc_f64_s', 0xb1: 'i64.trunc_f64_u', 0xb2: 'f32.conv_i32_s', 0xb3: 'f32.conv_i32_u',
      0xb4: 'f32.conv_i64_s', 0xb5: 'f32.conv_i64_u', 0xb6: 'f32.demote', 0xb7: 'f64.conv_i32_s',
      0xb8: 'f64.conv_i32_u', 0xb9: 'f64.conv_i64_s', 0xba: 'f64.conv_i64_u', 0xbb: 'f64.promote',
      0xbc: 'i32.reinterpret', 0xbd: 'i64.reinterpret', 0xbe: 'f32.reinterpret', 0xbf: 'f64.reinterpret',
      0xc0: 'ext8_s', 0xc1: 'ext16_s', 0xc2: 'ext8_s64', 0xc3: 'ext16_s64', 0xc4: 'ext32_s64'}
BIN_I = ['==', '!=', '<s', '<u', '>s', '>u', '<=s', '<=u', '>=s', '>=u']
BIN_F = ['==', '!=', '<', '>', '<=', '>=']
ARITH_I = ['+', '-', '*', '/s', '/u', '%s', '%u', '&', '|', '^', '<<', '>>s', '>>u', 'rotl', 'rotr']
ARITH_F = ['+', '-', '*', '/', 'min', 'max', 'copysign']


def binop(op):
    if 0x46 <= op <= 0x4f:
        return BIN_I[op - 0x46]
    if 0x51 <= op <= 0x5a:
        return BIN_I[op - 0x51] + '64'
    if 0x5b <= op <= 0x60:
        return BIN_F[op - 0x5b] + 'f'
    if 0x61 <= op <= 0x66:
        return BIN_F[op - 0x61] + 'd'
    if 0x6a <= op <= 0x78:
        return ARITH_I[op - 0x6a]
    if 0x7c <= op <= 0x8a:
        return ARITH_I[op - 0x7c] + '64'
    if 0x92 <= op <= 0x98:
        return ARITH_F[op - 0x92] + 'f'
    if 0xa0 <= op <= 0xa6:
        return ARITH_F[op - 0xa0] + 'd'
    return None


class Module:
    def __init__(self, path):
        self.b = open(path, 'rb').read()
        self.secs = sections(self.b)
        self._types()
        self._imports()
        self._funcs()
        self._exports()
        self._elems()
        self._globals()
        self._code()

    def _types(self):
        b = self.b
        i, _ = self.secs[1]
        n, i = uleb(b, i)
        self.types = []
        for _ in range(n):
            assert b[i] == 0x60
            np_, i = uleb(b, i + 1)
            ps = [VT[x] for x in b[i:i + np_]]
            i += np_
            nr, i = uleb(b, i)
            rs = [VT[x] for x in b[i:i + nr]]
            i += nr
            self.types.append((ps, rs))

    def _imports(self):
        b = self.b
        self.imports = []
        self.nfimp = 0
        self.func_type = []
        if 2 not in self.secs:
            return
        i, _ = self.secs[2]
        n, i = uleb(b, i)
        for _ in range(n):
            l, i = uleb(b, i)
            mod = b[i:i + l].decode()
            i += l
            l, i = uleb(b, i)
            nm = b[i:i + l].decode()
            i += l
            kind = b[i]
            i += 1
            if kind == 0:
                t, i = uleb(b, i)
                self.func_type.append(t)
                self.nfimp += 1
                self.imports.append((mod, nm, 'func', t))
            elif kind == 1:
                i += 1
                f = b[i]
                i += 1
                _, i = uleb(b, i)
                if f & 1:
                    _, i = uleb(b, i)
                self.imports.append((mod, nm, 'table', None))
            elif kind == 2:
                f = b[i]
                i += 1
                _, i = uleb(b, i)
                if f & 1:
                    _, i = uleb(b, i)
                self.imports.append((mod, nm, 'memory', f))
            elif kind == 3:
                i += 2
                self.imports.append((mod, nm, 'global', None))

    def _funcs(self):
        b = self.b
        i, _ = self.secs[3]
        n, i = uleb(b, i)
        for _ in range(n):
            t, i = uleb(b, i)
            self.func_type.append(t)

    def _exports(self):
        b = self.b
        self.exports = {}
        i, _ = self.secs[7]
        n, i = uleb(b, i)
        for _ in range(n):
            l, i = uleb(b, i)
            nm = b[i:i + l].decode()
            i += l
            kind = b[i]
            idx, i = uleb(b, i + 1)
            if kind == 0:
                self.exports[idx] = nm

    def _elems(self):
        """table slot -> function index (call_indirect targets: OpenH264's function pointers / vtables)"""
        b = self.b
        self.table = {}
        if 9 not in self.secs:
            return
        i, _ = self.secs[9]
        n, i = uleb(b, i)
        for _ in range(n):
            flag, i = uleb(b, i)
            assert flag == 0, flag
            assert b[i] == 0x41
            off, i = sleb(b, i + 1)
            assert b[i] == 0x0b
            i += 1
            cnt, i = uleb(b, i)
            for k in range(cnt):
                f, i = uleb(b, i)
                self.table[off + k] = f

    def _globals(self):
        self.nglob_imp = sum(1 for im in self.imports if im[2] == 'global')

    def _code(self):
        b = self.b
        i, _ = self.secs[10]
        n, i = uleb(b, i)
        self.bodies = []
        for _ in range(n):
            sz, i = uleb(b, i)
            self.bodies.append((i, sz))
            i += sz

    def body(self, f):
        return self.bodies[f - self.nfimp]

    def sig(self, f):
        return self.types[self.func_type[f]]


class Dis:
    """folds one function body into statements"""

    def __init__(self, m, f):
        self.m, self.f = m, f
        self.b = m.b
        self.out = []
        self.tmp = 0
        self.calls = []
        self.consts = []

    def emit(self, depth, s, off):
        self.out.append(f'{"  " * depth}{s:<90s} @{off}')

    def run(self):
        m, b = self.m, self.b
        start, size = m.body(self.f)
        end = start + size
        i = start
        nloc, i = uleb(b, i)
        ps, rs = m.sig(self.f)
        nlocals = len(ps)
        decl = []
        for _ in range(nloc):
            c, i = uleb(b, i)
            decl.append(f'{c}x{VT[b[i]]}')
            nlocals += c
            i += 1
        name = m.exports.get(self.f, '')
        self.out.append(f'func {self.f} {name} ({", ".join(ps)}) -> ({", ".join(rs)}) locals {" ".join(decl)} '
                        f'@{start}..{end}')
        stack = []
        ctl = []  # (kind, stack height, result arity)
        depth = 1

        def pop():
            return stack.pop() if stack else '<?>'

        def flush(d):
            # values still on the stack at a statement boundary are kept (wasm allows it); show them
            pass

        while i < end:
            off = i
            op = b[i]
            i += 1
            if op == 0x00:
                self.emit(depth, 'unreachable', off)
            elif op == 0x01:
                pass
            elif op in (0x02, 0x03, 0x04):
                bt = b[i]
                if bt == 0x40:
                    nres, i = 0, i + 1
                elif bt in VT:
                    nres, i = 1, i + 1
                else:
                    t, i = sleb(b, i)
                    nres = len(m.types[t][1])
                kw = {2: 'block', 3: 'loop', 4: 'if'}[op]
                if op == 0x04:
                    c = pop()
                    self.emit(depth, f'if ({c}) {{' + (f'  -> {nres}' if nres else ''), off)
                else:
                    self.emit(depth, f'{kw} B{len(ctl)} {{' + (f'  -> {nres}' if nres else ''), off)
                ctl.append((kw, len(stack), nres))
                depth += 1
            elif op == 0x05:
                kw, h, nres = ctl[-1]
                if nres and len(stack) > h:
                    self.emit(depth, f'yield {pop()}', off)
                del stack[h:]
                self.emit(depth - 1, '} else {', off)
            elif op == 0x0b:
                if not ctl:
                    if stack:
                        self.emit(depth, f'return {pop()}', off)
                    self.out.append('end')
                    break
                kw, h, nres = ctl.pop()
                vals = []
                if nres and len(stack) > h:
                    vals = [pop()]
                    self.emit(depth, f'yield {vals[0]}', off)
                del stack[h:]
                depth -= 1
                self.emit(depth, '}', off)
                if nres:
                    t = f'r{self.tmp}'
                    self.tmp += 1
                    stack.append(t)
                    self.emit(depth, f'{t} = <block result>', off)
            elif op == 0x0c:
                l, i = uleb(b, i)
                tgt = len(ctl) - 1 - l
                kw = ctl[tgt][0] if tgt >= 0 else 'func'
                carry = f' carry {stack[-1]}' if tgt >= 0 and kw != 'loop' and ctl[tgt][2] and stack else ''
                self.emit(depth, f'br B{tgt} ({kw}{"=continue" if kw == "loop" else ""}){carry}', off)
            elif op == 0x0d:
                l, i = uleb(b, i)
                c = pop()
                tgt = len(ctl) - 1 - l
                kw = ctl[tgt][0] if tgt >= 0 else 'func'
                carry = f' carry {stack[-1]}' if tgt >= 0 and kw != 'loop' and ctl[tgt][2] and stack else ''
                self.emit(depth, f'br_if ({c}) B{tgt} ({kw}{"=continue" if kw == "loop" else ""}){carry}', off)
            elif op == 0x0e:
                n, i = uleb(b, i)
                ls = []
                for _ in range(n + 1):
                    l, i = uleb(b, i)
                    ls.append(f'B{len(ctl) - 1 - l}')
                c = pop()
                self.emit(depth, f'br_table ({c}) [{", ".join(ls[:-1])}] default {ls[-1]}', off)
            elif op == 0x0f:
                if rs and stack:
                    self.emit(depth, f'return {pop()}', off)
                else:
                    self.emit(depth, 'return', off)
            elif op == 0x10:
                fi, i = uleb(b, i)
                ps2, rs2 = m.sig(fi)
                args = [pop() for _ in ps2][::-1]
                nm = m.exports.get(fi, '')
                imp = m.imports[fi][1] if fi < m.nfimp else ''
                label = f'f{fi}' + (f'<{nm}>' if nm else '') + (f'<import:{imp}>' if imp else '')
                self.calls.append(fi)
                call = f'{label}({", ".join(args)})'
                if rs2:
                    t = f't{self.tmp}'
                    self.tmp += 1
                    self.emit(depth, f'{t} = {call}', off)
                    stack.append(t)
                else:
                    self.emit(depth, call, off)
            elif op == 0x11:
                ti, i = uleb(b, i)
                _, i = uleb(b, i)
                ps2, rs2 = m.types[ti]
                idx = pop()
                args = [pop() for _ in ps2][::-1]
                call = f'icall<t{ti}>[{idx}]({", ".join(args)})'
                if rs2:
                    t = f't{self.tmp}'
                    self.tmp += 1
                    self.emit(depth, f'{t} = {call}', off)
                    stack.append(t)
                else:
                    self.emit(depth, call, off)
            elif op == 0x1a:
                v = pop()
                if v.startswith('t') or v.startswith('r'):
                    pass
                else:
                    self.emit(depth, f'drop {v}', off)
            elif op == 0x1b:
                c = pop()
                y = pop()
                x = pop()
                stack.append(f'({c} ? {x} : {y})')
            elif op == 0x1c:
                n, i = uleb(b, i)
                i += n
                c = pop()
                y = pop()
                x = pop()
                stack.append(f'({c} ? {x} : {y})')
            elif op == 0x20:
                x, i = uleb(b, i)
                stack.append(f'L{x}')
            elif op in (0x21, 0x22):
                x, i = uleb(b, i)
                v = pop()
                # pending stack values that read the old value of L{x} are snapshotted first
                pat = re.compile(rf'\bL{x}\b')
                for k, e in enumerate(stack):
                    if pat.search(e):
                        t = f's{self.tmp}'
                        self.tmp += 1
                        self.emit(depth, f'{t} = {e}', off)
                        stack[k] = t
                self.emit(depth, f'L{x} = {v}', off)
                if op == 0x22:
                    stack.append(f'L{x}')
            elif op == 0x23:
                x, i = uleb(b, i)
                stack.append(f'G{x}')
            elif op == 0x24:
                x, i = uleb(b, i)
                self.emit(depth, f'G{x} = {pop()}', off)
            elif op in LOADS:
                _, i = uleb(b, i)
                o, i = uleb(b, i)
                a = pop()
                stack.append(f'{LOADS[op][0]}[{a}{"+" + str(o) if o else ""}]')
            elif op in STORES:
                _, i = uleb(b, i)
                o, i = uleb(b, i)
                v = pop()
                a = pop()
                self.emit(depth, f'{STORES[op]}[{a}{"+" + str(o) if o else ""}] = {v}', off)
            elif op == 0x3f:
                i += 1
                stack.append('memory.size')
            elif op == 0x40:
                i += 1
                stack.append(f'memory.grow({pop()})')
            elif op == 0x41:
                v, i = sleb(b, i)
                v = (v + (1 << 31)) % (1 << 32) - (1 << 31)
                self.consts.append((off, v))
                stack.append(str(v))
            elif op == 0x42:
                v, i = sleb(b, i)
                stack.append(f'{v}L')
            elif op == 0x43:
                v = struct.unpack_from('<f', b, i)[0]
                i += 4
                stack.append(f'{v!r}f')
            elif op == 0x44:
                v = struct.unpack_from('<d', b, i)[0]
                i += 8
                stack.append(f'{v!r}d')
            elif op in UN:
                stack.append(f'{UN[op]}({pop()})')
            elif binop(op):
                y = pop()
                x = pop()
                stack.append(f'({x} {binop(op)} {y})')
            elif op == 0xfc:
                sub, i = uleb(b, i)
                if sub <= 7:
                    stack.append(f'trunc_sat{sub}({pop()})')
                elif sub == 8:
                    seg, i = uleb(b, i)
                    i += 1
                    n_ = pop()
                    s_ = pop()
                    d_ = pop()
                    self.emit(depth, f'memory.init(seg {seg}, dst {d_}, src {s_}, n {n_})', off)
                elif sub == 9:
                    _, i = uleb(b, i)
                elif sub == 10:
                    i += 2
                    n_ = pop()
                    s_ = pop()
                    d_ = pop()
                    self.emit(depth, f'memcpy({d_}, {s_}, {n_})', off)
                elif sub == 11:
                    i += 1
                    n_ = pop()
                    v_ = pop()
                    d_ = pop()
                    self.emit(depth, f'memset({d_}, {v_}, {n_})', off)
                else:
                    raise ValueError(f'0xfc {sub} at {off}')
            elif op == 0xfd:
                sub, i = uleb(b, i)
                if sub <= 11 or 92 <= sub <= 93:
                    _, i = uleb(b, i)
                    o, i = uleb(b, i)
                    if sub == 11:
                        v = pop()
                        a = pop()
                        self.emit(depth, f'v128[{a}+{o}] = {v}', off)
                    else:
                        stack.append(f'v128load{sub}[{pop()}+{o}]')
                elif sub == 12:
                    i += 16
                    stack.append('v128.const')
                elif sub == 13:
                    i += 16
                    y = pop()
                    x = pop()
                    stack.append(f'shuffle({x},{y})')
                elif 21 <= sub <= 34:
                    lane = b[i]
                    i += 1
                    if sub in (23, 26, 28, 30, 32, 34):
                        v = pop()
                        x = pop()
                        stack.append(f'replace_lane{sub}({x},{lane},{v})')
                    else:
                        stack.append(f'extract_lane{sub}({pop()},{lane})')
                elif 84 <= sub <= 91:
                    raise ValueError(f'simd lane load/store at {off}')
                else:
                    # generic simd op: guess arity by common cases (splat: 1; binary arith: 2)
                    if 15 <= sub <= 20:
                        stack.append(f'splat{sub}({pop()})')
                    else:
                        y = pop()
                        x = pop()
                        stack.append(f'simd{sub}({x},{y})')
            elif op == 0xfe:
                sub, i = uleb(b, i)
                if sub == 3:
                    i += 1
                    self.emit(depth, 'atomic.fence', off)
                else:
                    _, i = uleb(b, i)
                    o, i = uleb(b, i)
                    # atomics: notify(0: addr,count) wait32/64 (1,2: addr,expected,timeout), loads 0x10-0x16,
                    # stores 0x17-0x1d, rmw 0x1e-0x4e
                    if sub == 0:
                        c = pop()
                        a = pop()
                        t = f't{self.tmp}'
                        self.tmp += 1
                        self.emit(depth, f'{t} = atomic.notify({a}+{o}, {c})', off)
                        stack.append(t)
                    elif sub in (1, 2):
                        to = pop()
                        ex = pop()
                        a = pop()
                        t = f't{self.tmp}'
                        self.tmp += 1
                        self.emit(depth, f'{t} = atomic.wait({a}+{o}, {ex}, {to})', off)
                        stack.append(t)
                    elif 0x10 <= sub <= 0x16:
                        stack.append(f'atomic_load{sub}[{pop()}+{o}]')
                    elif 0x17 <= sub <= 0x1d:
                        v = pop()
                        a = pop()
                        self.emit(depth, f'atomic_store{sub}[{a}+{o}] = {v}', off)
                    elif 0x48 <= sub <= 0x4e:
                        r = pop()
                        e_ = pop()
                        a = pop()
                        t = f't{self.tmp}'
                        self.tmp += 1
                        self.emit(depth, f'{t} = atomic_cmpxchg{sub}({a}+{o}, {e_}, {r})', off)
                        stack.append(t)
                    else:
                        v = pop()
                        a = pop()
                        t = f't{self.tmp}'
                        self.tmp += 1
                        self.emit(depth, f'{t} = atomic_rmw{sub}({a}+{o}, {v})', off)
                        stack.append(t)
            else:
                raise ValueError(f'opcode {op:#x} at {off} in func {self.f}')
        return self.out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--wasm', default=DEFAULT_WASM)
    ap.add_argument('--out', default='/tmp/wasm_dis')
    ap.add_argument('--func', type=int, nargs='*')
    a = ap.parse_args()
    m = Module(a.wasm)
    os.makedirs(a.out, exist_ok=True)
    funcs = a.func or range(m.nfimp, m.nfimp + len(m.bodies))
    callers = {}
    with open(os.path.join(a.out, 'all.txt'), 'w') as fa:
        for f in funcs:
            d = Dis(m, f)
            lines = d.run()
            fa.write('\n'.join(lines) + '\n\n')
            for c in d.calls:
                callers.setdefault(c, set()).add(f)
    with open(os.path.join(a.out, 'callers.txt'), 'w') as fc:
        for c in sorted(callers):
            fc.write(f'{c}: {sorted(callers[c])}\n')
    with open(os.path.join(a.out, 'table.txt'), 'w') as ft:
        for k in sorted(m.table):
            ft.write(f'{k}: f{m.table[k]}\n')
    print(f'{len(list(funcs))} functions -> {a.out}/all.txt; exports {m.exports}')


if __name__ == '__main__':
    main()
