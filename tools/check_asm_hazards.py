"""Static audit of the asm-MFMA kernels (gemm_big.hip gemm_w4_kernel*): hipcc pads no hazards for
an inline-asm MFMA (cdna_hip_programming.md §5.7 item 2), so check the emitted ISA for
  1. a VALU instruction writing a VGPR that the next MFMA reads as A/B within 2 wait states
     (an `s_nop N` or intervening instructions count as N+1 / 1 states each),
  2. compiler v_accvgpr_{write,mov} to an accumulator AGPR between the first and the last MFMA
     (an accumulator shuttled or clobbered outside the asm chain),
  3. a v_accvgpr_read of an AGPR within 12 states of the MFMA that wrote it (8-pass XDL -> reader),
  4. scratch (spills) inside the MFMA span.
Usage: python tools/check_asm_hazards.py file.s [kernel-substring]   (exit 1 on findings)
"""
import re
import sys


def regs(tok):
    """'v[4:7]' -> {4..7}; 'v12' -> {12}; for one register file prefix."""
    m = re.match(r'([va])\[(\d+):(\d+)\]', tok)
    if m:
        return m.group(1), set(range(int(m.group(2)), int(m.group(3)) + 1))
    m = re.match(r'([va])(\d+)$', tok)
    if m:
        return m.group(1), {int(m.group(2))}
    return None, set()


def audit(lines, name):
    insts = []
    for l in lines:
        t = l.strip()
        if not t or t.startswith(';') or t.startswith('.') or t.endswith(':'):
            continue
        insts.append(t.split(';')[0].strip())
    problems = []
    mf = [i for i, t in enumerate(insts) if t.startswith('v_mfma')]
    if not mf:
        return problems
    for k, i in enumerate(mf):
        ops = [o.strip() for o in insts[i].split(None, 1)[1].split(',')]
        srcab = set()
        for o in ops[1:3]:
            f, r = regs(o)
            if f == 'v':
                srcab |= r
        states = 0
        j = i - 1
        while j >= 0 and states < 2:
            t = insts[j]
            if t.startswith('s_nop'):
                states += int(t.split()[1]) + 1
                j -= 1
                continue
            if t.startswith('v_') and not t.startswith('v_mfma') and not t.startswith('v_accvgpr_read'):
                dst = t.split(None, 1)[1].split(',')[0].strip() if ' ' in t else ''
                f, r = regs(dst)
                if f == 'v' and r & srcab:
                    problems.append(f'{name}: VALU -> MFMA operand hazard: "{t}" then "{insts[i]}"')
            states += 1
            j -= 1
    first, last = mf[0], mf[-1]
    for i in range(first, last):
        t = insts[i]
        if t.startswith('v_accvgpr_write') or t.startswith('v_accvgpr_mov'):
            problems.append(f'{name}: accumulator write inside the MFMA span: "{t}"')
        if t.startswith('scratch_') or t.startswith('buffer_store') and 'off' in t:
            problems.append(f'{name}: scratch access inside the MFMA span: "{t}"')
    # MFMA D -> v_accvgpr_read within 12 states
    for i in mf:
        d = insts[i].split(None, 1)[1].split(',')[0].strip()
        f, dr = regs(d)
        states, j = 0, i + 1
        while j < len(insts) and states < 12:
            t = insts[j]
            if t.startswith('s_nop'):
                states += int(t.split()[1]) + 1
                j += 1
                continue
            if t.startswith('v_accvgpr_read'):
                src = t.split(',')[1].strip()
                f2, r2 = regs(src)
                if f2 == 'a' and r2 & dr:
                    problems.append(f'{name}: MFMA D read after {states} states: "{insts[i]}" then "{t}"')
            states += 1
            j += 1
    return problems


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else 'gemm_w4_kernel'
    s = open(path).read()
    probs, n = [], 0
    for m in re.finditer(r'^(_Z[^:\s]*' + re.escape(pat) + r'[^:\s]*):', s, re.M):
        name = m.group(1)
        end = s.index('.Lfunc_end', m.end())
        probs += audit(s[m.end():end].split('\n'), name)
        n += 1
    for p in probs[:40]:
        print(p)
    print(f'{n} kernels audited, {len(probs)} findings')
    sys.exit(1 if probs or n == 0 else 0)


if __name__ == '__main__':
    main()
