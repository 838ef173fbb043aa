"""Check of the split-bf16 M-split kernels' asm MFMAs (fc_common.h P<BF16X3>::mma_a / mma_a2, which hipcc's hazard
recognizer does not see into): in the device assembly, no instruction other than a dependent MFMA may touch an MFMA's
destination within 12 wait states (approximated as 1 per instruction, N + 1 per s_nop N).  The gfx950 requirement
for a 4-pass XDL MFMA (v_mfma_f32_16x16x32_bf16: 16 cycles, PMC) writing a VGPR that a VALU then reads is 7 wait
states; mma_fence pads 12.  Run by tests/test_hazard_check.py on every build (CPU), or by hand:
    hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -fno-slp-vectorize -Iinclude \
        -Ihumanoid_mppi-rl_amd/csrc humanoid_mppi-rl_amd/csrc/kernels_fc_ca.hip -o /tmp/ca.s
    python tools/mfma_hazard_check.py /tmp/ca.s"""
import re
import sys

KERNELS = r'^(_ZN4mppi21fc_rollout_kernel_x3w\w+|_ZN4mppi20fc_rollout_kernel_x3I\w+|_ZN4mppi21fc_rollout_kernel_x3[dh]\w+):'
WAIT_STATES = 12


def regs(tok):
    m = re.match(r'([va])\[(\d+):(\d+)\]', tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r'([va])(\d+)$', tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def check(s, pattern=KERNELS, verbose=False):
    """[(kernel symbol, asm MFMA count, flagged accesses)] for every kernel of the assembly text `s` matching
    `pattern`.  Only MFMAs from inline asm (between the compiler's ;;#ASMSTART / ;;#ASMEND markers) are checked: the
    hazard recognizer pads the ones the compiler selects itself."""
    out = []
    for name in re.findall(pattern, s, re.M):
        i = s.find(name + ':')
        j = s.find('s_endpgm', i)
        lines, in_asm = [], []
        asm = False
        for ln in s[i:j].split('\n'):
            t = ln.strip()
            if t.startswith(';;#ASMSTART'):
                asm = True
            elif t.startswith(';;#ASMEND'):
                asm = False
            elif t and not t.startswith(';') and not t.startswith('.'):
                lines.append(t)
                in_asm.append(asm)
        bad = 0
        n_mfma = 0
        for k, ln in enumerate(lines):
            if not ln.startswith('v_mfma') or not in_asm[k]:
                continue
            n_mfma += 1
            dst = regs(ln.split()[1].rstrip(','))
            ws = 0
            for l2 in lines[k + 1:k + 40]:
                op = l2.split()[0]
                if op == 's_nop':
                    ws += int(l2.split()[1], 0) + 1
                elif op.startswith('v_mfma'):
                    toks = [t.rstrip(',') for t in l2.split()[1:]]
                    # dependent accumulate (srcC == dst exactly) is fine; any other overlap is flagged
                    if dst & (regs(toks[1]) | regs(toks[2])):
                        bad += 1
                        if verbose:
                            print('MFMA src overlap', ln, '->', l2)
                    ws += 1
                else:
                    toks = [t.rstrip(',') for t in l2.split()[1:]]
                    if any(dst & regs(t) for t in toks) and ws < WAIT_STATES:
                        bad += 1
                        if verbose:
                            print('early access', ws, ln, '->', l2)
                    ws += 1
                if ws >= WAIT_STATES:
                    break
        out.append((name, n_mfma, bad))
    return out


if __name__ == '__main__':
    for name, n, bad in check(open(sys.argv[1]).read(), verbose=True):
        print(name[12:45], 'mfma', n, 'flagged', bad)
