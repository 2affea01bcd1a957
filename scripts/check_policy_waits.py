"""Check the counted waits of k_policy_train_db in the built library's ISA
(ADVICE r04): each land_db<NST> (mas_policy.hip) waits with vmcnt(min(NST,
63)) for the LDS-DMA copies of the next weight stage, which is only correct
if at least that many vector memory instructions were issued after those
copies (vmcnt retires in issue order; a wave holds at most 63).  The copies
are inline asm the compiler does not count, so nothing else verifies it: a
load the compiler merged (two 2-B loads into one 4-B load) would silently
make a hand count too high.  land_db marks itself with `s_movk_i32 sX,
0x7a00 + n`; for every marker this script counts the VMEM instructions
between the last `global_load_lds_dwordx4` before it and the marker.
usage: python scripts/check_policy_waits.py [libmas.so]   (exit 1 on a violation)"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'gym-ma-survival-2d_amd', 'masurvival', '_lib', 'libmas.so')
OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'
VMEM = re.compile(r'^\s*(global_load|global_store|global_atomic|buffer_load|buffer_store|buffer_atomic|'
                  r'scratch_load|scratch_store|flat_load|flat_store|flat_atomic)')
MARK = re.compile(r's_movk_i32\s+s\d+,\s*0x7a([0-9a-f]{2})')


def disassemble(lib):
    """The device code objects of lib (gfx950), disassembled."""
    out = []
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


def check(asm):
    """[(kernel, marker n, VMEM ops since the last copy)] and the violations."""
    lines = asm.split('\n')
    rows, bad, kern = [], [], None
    since = None
    for l in lines:
        m = re.match(r'^[0-9a-f]+ <(.*)>:', l)
        if m:
            kern = m.group(1) if 'k_policy_train_db' in m.group(1) else None
            since = None
            continue
        if kern is None:
            continue
        ins = l.split('//')[0].strip()
        if ins.startswith('global_load_lds_dwordx4'):
            since = 0
            continue
        if since is not None and VMEM.match(ins):
            since += 1
        mk = MARK.search(ins)
        if mk:
            n = int(mk.group(1), 16)
            got = since if since is not None else 0
            rows.append((kern, n, got))
            if n > 0 and got < n:
                bad.append((kern, n, got))
    return rows, bad


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else LIB
    rows, bad = check(disassemble(lib))
    if not rows:
        print('check_policy_waits: no land_db markers found in', lib)
        return 1
    for k, n, got in rows:
        print(f'{k[:60]:60s} wait n={n:2d}  VMEM after the copies: {got}')
    if bad:
        print('check_policy_waits: VIOLATION -- a counted wait exceeds the operations issued after its copies:', bad)
        return 1
    print(f'check_policy_waits: {len(rows)} counted waits OK')
    return 0


if __name__ == '__main__':
    sys.exit(main())
