"""Check the counted waits of k_policy_train_db in the built library's ISA
(ADVICE r04): each land_db<NST> (mas_policy.hip) waits with vmcnt(min(NST,
63)) for the LDS-DMA copies of the next weight stage, which is only correct
if at least that many vector memory instructions were issued after those
copies (vmcnt retires in issue order; a wave holds at most 63).  The copies
are inline asm the compiler does not count, so nothing else verifies it: a
load the compiler merged (two 2-B loads into one 4-B load) would silently
make a hand count too high.  land_db marks itself with `s_movk_i32 sX,
0x7a00 + n`; for every marker this script counts the VMEM instructions
on every path from the last `global_load_lds_dwordx4` to the marker: a
forward dataflow over the kernel's branches (s_branch / s_cbranch_*) takes
the minimum count over a branch target's predecessors, back edges included,
iterated to a fixed point, so a marker reached over a loop back edge or a
branch that skips some VMEM ops is checked against its fewest.
llvm-objdump comes from $ROCM_PATH (default /opt/rocm), or from hipconfig.
usage: python scripts/check_policy_waits.py [libmas.so]   (exit 1 on a violation)"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'gym-ma-survival-2d_amd', 'masurvival', '_lib', 'libmas.so')


def find_objdump():
    """llvm-objdump of the ROCm install: $ROCM_PATH, else hipconfig's, else /opt/rocm."""
    roots = [os.environ.get('ROCM_PATH')]
    hc = shutil.which('hipconfig')
    if hc:
        try:
            roots.append(subprocess.run([hc, '--rocmpath'], capture_output=True, text=True, check=True).stdout.strip())
        except (OSError, subprocess.CalledProcessError):
            pass
    roots.append('/opt/rocm')
    for r in roots:
        if r and os.path.exists(os.path.join(r, 'lib', 'llvm', 'bin', 'llvm-objdump')):
            return os.path.join(r, 'lib', 'llvm', 'bin', 'llvm-objdump')
    raise FileNotFoundError('check_policy_waits: llvm-objdump not found under $ROCM_PATH, hipconfig --rocmpath or '
                            '/opt/rocm (lib/llvm/bin/llvm-objdump); set ROCM_PATH')


VMEM = re.compile(r'^\s*(global_load|global_store|global_atomic|buffer_load|buffer_store|buffer_atomic|'
                  r'scratch_load|scratch_store|flat_load|flat_store|flat_atomic)')
MARK = re.compile(r's_movk_i32\s+s\d+,\s*0x7a([0-9a-f]{2})')


def disassemble(lib):
    """The device code objects of lib (gfx950), disassembled."""
    out = []
    OBJDUMP = find_objdump()
    with tempfile.TemporaryDirectory() as d:
        dst = os.path.join(d, 'lib.so')
        shutil.copy(lib, dst)
        subprocess.run([OBJDUMP, '--offloading', dst], cwd=d, check=True, capture_output=True)
        for f in sorted(os.listdir(d)):
            if 'gfx950' in f:
                r = subprocess.run([OBJDUMP, '-d', '--mcpu=gfx950', os.path.join(d, f)], check=True,
                                   capture_output=True, text=True)
                out.append(r.stdout)
    return '\n'.join(out)


BRANCH = re.compile(r'^s_(c?branch\w*)\s+(-?\d+)')
WAIT = re.compile(r'^s_waitcnt\b.*\bvmcnt\((\d+)\)')
ADDR = re.compile(r'//\s*([0-9A-Fa-f]+):')
NO_FALL = ('s_branch', 's_endpgm', 's_setpc_b64')
SAFE = 1 << 20  # no copy outstanding on this path (none issued yet, or an earlier wait completed it)


def check(asm):
    """[(kernel, marker n, VMEM ops since the last copy on its worst path)] and
    the violations.  Per kernel, a forward dataflow over the instructions:
    in(i) = min(out(fall-through predecessor), out(each branch to i)),
    out(i) = 0 after a copy, +1 after a VMEM op, SAFE after an
    `s_waitcnt vmcnt(m)` with m <= the count (the copies have landed), else
    in(i); iterated to a fixed point (values only decrease).  Path-insensitive:
    a path the kernel cannot take still counts, so the source keeps every
    counted wait on paths that all carry its stores."""
    kernels, kern = [], None
    for l in asm.split('\n'):
        m = re.match(r'^[0-9a-f]+ <(.*)>:', l)
        if m:
            kern = [m.group(1), []] if 'k_policy_train_db' in m.group(1) else None
            if kern:
                kernels.append(kern)
            continue
        if kern is None:
            continue
        ins = l.split('//')[0].strip()
        a = ADDR.search(l)
        if ins and a:
            kern[1].append((int(a.group(1), 16), ins))
    rows, bad = [], []
    INF = 1 << 30
    for name, code in kernels:
        at = {addr: k for k, (addr, _) in enumerate(code)}
        preds = [[] for _ in code]  # branch sources per target index
        for k, (addr, ins) in enumerate(code):
            b = BRANCH.match(ins)
            if b:
                tgt = addr + 4 + 4 * int(b.group(2))
                if tgt in at:
                    preds[at[tgt]].append(k)
        out = [INF] * len(code)
        changed = True
        while changed:
            changed = False
            for k, (addr, ins) in enumerate(code):
                cand = [SAFE] if k == 0 else []
                if k > 0 and not code[k - 1][1].startswith(NO_FALL):
                    cand.append(out[k - 1])
                cand += [out[j] for j in preds[k]]
                v = min(cand) if cand else INF
                w = WAIT.match(ins)
                if ins.startswith('global_load_lds_dwordx4'):
                    v = 0
                elif v < SAFE and VMEM.match(ins):
                    v += 1
                elif v < SAFE and w and int(w.group(1)) <= v:
                    v = SAFE
                if v < out[k]:
                    out[k] = v
                    changed = True
        for k, (addr, ins) in enumerate(code):
            mk = MARK.search(ins)
            if mk:
                n = int(mk.group(1), 16)
                # the marker's own count is its in-state (it is no VMEM op)
                # (in-state: the fall-through predecessor's out, or a branch's)
                ins_k = [out[k - 1]] if k > 0 and not code[k - 1][1].startswith(NO_FALL) else []
                ins_k += [out[j] for j in preds[k]]
                got = min(ins_k) if ins_k else SAFE
                got = got if got < INF else 0
                rows.append((name, n, got))
                if n > 0 and got < n:
                    bad.append((name, n, got))
    return rows, bad


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else LIB
    rows, bad = check(disassemble(lib))
    if not rows:
        print('check_policy_waits: no land_db markers found in', lib)
        return 1
    for k, n, got in rows:
        g = 'copies landed' if got >= SAFE else f'VMEM after the copies: {got}'
        print(f'{k[:60]:60s} wait n={n:2d}  {g}')
    if bad:
        print('check_policy_waits: VIOLATION -- a counted wait exceeds the operations issued after its copies:', bad)
        return 1
    print(f'check_policy_waits: {len(rows)} counted waits OK')
    return 0


if __name__ == '__main__':
    sys.exit(main())
