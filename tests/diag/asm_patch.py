"""Diagnostic: pad a kernel's gfx950 assembly with extra wait states by hazard class, to
bisect schedule-dependent wrong results (tests/diag/build_asm.sh assembles the output).

    python tests/diag/asm_patch.py POLICY in.s out.s [STATES]

POLICY: none | allmfma (STATES after every MFMA) | raw (non-MFMA reader of an MFMA result)
        | trans (any reader of a transcendental's result; tpk / tmfma / tother: only v_pk_* /
        MFMA / other VALU readers) | valuraw (VALU reader of a VALU
        result) | war (non-MFMA writer of a register an MFMA read; warv: VMEM loads excluded) | valu2mfma (MFMA reading a
        register a non-MFMA wrote) — each pads the instruction pair to at least STATES
        (default 24) wait states.  Counting is straight-line (labels do not reset it).
        Waitcnt rewrites (DESIGN.md §7.1 bisection): vm0 / lgkm0 turn every compiler-emitted
        partial vmcnt / lgkmcnt wait into a full one, exp0 adds expcnt(0) to every s_waitcnt.
        After-class inserts: wz_<cls> puts a full s_waitcnt 0 after, nop_<cls> an s_nop 0 after,
        every instruction of class cls = all | vload | vstore | lds | smem | valu | mfma (wz_all
        restates -amdgpu-waitcnt-forcezero on the assembly).
        swar: pad STATES wait states between a vector store of more than 8 bytes and a later
        writer of its data VGPRs (the GFX9 store-data hazard, which LLVM's hazard recognizer
        skips for MUBUF stores with an SGPR soffset).
"""
import re
import sys


def regs(tok):
    m = re.match(r'([va])\[(\d+):(\d+)\]', tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r'([va])(\d+)$', tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


TRANS = ('v_exp_f32', 'v_log_f32', 'v_rcp_f32', 'v_rsq_f32', 'v_sqrt_f32', 'v_sin_f32',
         'v_cos_f32')
NO_DST = ('buffer_store', 'global_store', 'scratch_store', 'ds_write', 's_', 'exp ')


def main():
    policy, src, dst = sys.argv[1:4]
    need = int(sys.argv[4]) if len(sys.argv) > 4 else 24
    out = []
    mfma_w, mfma_r, other_w = {}, {}, {}    # reg -> states since
    trans_w, valu_w = {}, {}
    inserted = 0

    def age(n):
        for d in (mfma_w, mfma_r, other_w, trans_w, valu_w):
            for r in d:
                d[r] += n

    if policy.startswith(('wz_', 'nop_')):
        kind, cls = policy.split('_', 1)
        ins = '\ts_waitcnt vmcnt(0) expcnt(0) lgkmcnt(0)\n' if kind == 'wz' else '\ts_nop 0\n'
        n, meta = 0, False
        for line in open(src):
            out.append(line)
            s = line.strip()
            meta = (meta or s.startswith('.amdgpu_metadata')) and \
                not s.startswith('.end_amdgpu_metadata')
            if meta or not s or s[0] in ';.' or s.endswith(':') or line[0] not in ' \t':
                continue
            op = s.split()[0]
            hit = {'all': not op.startswith(('s_endpgm', 's_setpc', 's_branch', 's_cbranch')),
                   'vload': op.startswith(('buffer_load', 'global_load', 'scratch_load')),
                   'vstore': op.startswith(('buffer_store', 'global_store', 'scratch_store',
                                            'buffer_atomic', 'global_atomic')),
                   'lds': op.startswith('ds_'),
                   'smem': op.startswith(('s_load', 's_buffer_load')),
                   'valu': op.startswith('v_') and not op.startswith('v_mfma'),
                   'mfma': op.startswith('v_mfma')}[cls]
            if hit:
                out.append(ins)
                n += 1
        open(dst, 'w').writelines(out)
        print('%s: %d inserted' % (policy, n))
        return
    if policy == 'swar':
        pending, n = {}, 0          # data reg -> states since the store
        for line in open(src):
            s = line.strip()
            if not s or s[0] in ';.' or s.endswith(':') or line[0] not in ' \t':
                out.append(line)
                continue
            parts = s.split(';')[0].replace(',', ' ').split()
            op, ops = parts[0], parts[1:]
            dst_regs = set() if op.startswith(NO_DST) or not ops else regs(ops[0])
            pad = max([need - pending[r] for r in dst_regs if r in pending] + [0])
            if pad > 0:
                out.append('\ts_nop %d\n' % (pad - 1))
                n += 1
                pending = {r: v + pad for r, v in pending.items()}
            out.append(line)
            k = int(ops[0], 0) + 1 if op == 's_nop' else 1
            pending = {r: v + k for r, v in pending.items() if v + k < need}
            if op.startswith(('buffer_store_dwordx3', 'buffer_store_dwordx4',
                              'global_store_dwordx3', 'global_store_dwordx4')):
                for r in regs(ops[0]):
                    pending[r] = 0
        open(dst, 'w').writelines(out)
        print('%s: %d pads inserted' % (policy, n))
        return
    if policy in ('vm0', 'lgkm0', 'exp0'):
        n = 0
        for line in open(src):
            st = line.strip()
            if st.startswith('s_waitcnt ') and not line.startswith(';'):
                new = line
                if policy == 'vm0':
                    new = re.sub(r'vmcnt\(\d+\)', 'vmcnt(0)', line)
                elif policy == 'lgkm0':
                    new = re.sub(r'lgkmcnt\(\d+\)', 'lgkmcnt(0)', line)
                elif 'expcnt' not in line:
                    new = line.rstrip('\n') + ' expcnt(0)\n'
                n += new != line
                line = new
            out.append(line)
        open(dst, 'w').writelines(out)
        print('%s: %d waits rewritten' % (policy, n))
        return
    for line in open(src):
        s = line.strip()
        is_ins = bool(s) and s[0] not in ';.' and not s.endswith(':') and line[0] in ' \t'
        if not is_ins:
            out.append(line)
            continue
        parts = s.split(';')[0].replace(',', ' ').split()
        op, ops = parts[0], parts[1:]
        mf = op.startswith('v_mfma')
        if mf:
            dst_regs = regs(ops[0]) if ops else set()
            src_regs = set().union(*[regs(t) for t in ops[1:4]]) if len(ops) > 1 else set()
        elif op.startswith(NO_DST):
            dst_regs = set()
            src_regs = set().union(*[regs(t) for t in ops]) if ops else set()
        else:
            dst_regs = regs(ops[0]) if ops else set()
            src_regs = set().union(*[regs(t) for t in ops[1:]]) if len(ops) > 1 else set()
        pad = 0
        if policy == 'raw' and not mf:
            for r in src_regs | dst_regs:
                if r in mfma_w:
                    pad = max(pad, need - mfma_w[r])
        elif policy in ('war', 'warv') and not mf and not (
                policy == 'warv' and op.startswith(('buffer_load', 'global_load'))):
            for r in dst_regs:
                if r in mfma_r:
                    pad = max(pad, need - mfma_r[r])
        elif policy == 'trans' or (policy == 'tpk' and op.startswith('v_pk_')) or (
                policy == 'tmfma' and mf) or (
                policy == 'tother' and op.startswith('v_') and not mf and not op.startswith('v_pk_')):
            for r in src_regs:
                if r in trans_w:
                    pad = max(pad, need - trans_w[r])
        elif policy == 'valuraw' and op.startswith('v_'):
            for r in src_regs:
                if r in valu_w:
                    pad = max(pad, need - valu_w[r])
        elif policy == 'valu2mfma' and mf:
            for r in src_regs:
                if r in other_w:
                    pad = max(pad, need - other_w[r])
        if pad > 0:
            inserted += 1
            age(pad)
            while pad > 0:
                k = min(pad, 16)
                out.append('\ts_nop %d\n' % (k - 1))
                pad -= k
        out.append(line)
        n = int(ops[0], 0) + 1 if op == 's_nop' else 1
        age(n)
        if mf:
            for r in dst_regs:
                mfma_w[r] = 0
            for r in src_regs:
                mfma_r[r] = 0
        else:
            for r in dst_regs:
                other_w[r] = 0
                mfma_w.pop(r, None)
                trans_w.pop(r, None)
                valu_w.pop(r, None)
                if op.startswith(TRANS):
                    trans_w[r] = 0
                if op.startswith('v_'):
                    valu_w[r] = 0
        for d in (mfma_w, mfma_r, other_w, trans_w, valu_w):
            for r in [r for r, v in d.items() if v > 64]:
                del d[r]
        if policy == 'allmfma' and mf:
            out.append('\ts_nop 15\n' * (need // 16) + ('\ts_nop %d\n' % (need % 16 - 1) if need % 16 else ''))
            age(need)
            inserted += 1
    open(dst, 'w').writelines(out)
    print('%s: %d pads inserted' % (policy, inserted))


if __name__ == '__main__':
    main()
