"""Static checks of SGPR spills to VGPR lanes in one kernel of a gfx950 assembly file
(`hipcc --cuda-device-only -S`), used for DESIGN.md §7 (the round-4/5 k_mcmc_scan<TD> fault) and
§6 (spill reloads inside the headline kernel's iteration loop).

    python scripts/spill_flow.py FILE.s KERNEL_SYMBOL_PREFIX [--all]

Reports
  * the spill VGPRs (targets of v_writelane_b32) and every other instruction that writes one of
    them (a VALU write to a spill VGPR under a partial EXEC would clobber live spill lanes);
  * a reaching-definition analysis over the kernel's CFG for every spill slot (VGPR, lane):
    for each v_readlane_b32 of a slot, the v_writelane_b32 instructions that reach it (more
    than one is a loop or branch phi of one quantity, or a slot-sharing error — listed for
    inspection; --all lists every read);
  * spill reloads / stores per loop (by the assembler's loop annotations).
"""
import re
import sys
from collections import Counter, defaultdict


def extract(path, prefix):
    src = open(path).read().split('\n')
    start = None
    for i, l in enumerate(src):
        if start is None and re.match(r'^' + re.escape(prefix) + r'\S*:', l):
            start = i
        elif start is not None and l.startswith('.Lfunc_end'):
            return src[start:i + 1]
    raise SystemExit(f"no function {prefix}* in {path}")


def cfg(L):
    blocks = []
    for i, l in enumerate(L):
        m = re.match(r'^(\.LBB\d+_\d+):', l) or re.match(r'^; %bb\.(\d+):', l)
        if m:
            blocks.append([m.group(1) if l.startswith('.') else '%bb.' + m.group(1), i, None])
        elif i == 0:
            blocks.append(['entry', i, None])
    for k in range(len(blocks)):
        blocks[k][2] = blocks[k + 1][1] if k + 1 < len(blocks) else len(L)
    idx = {b[0]: k for k, b in enumerate(blocks)}
    succ, insts = defaultdict(list), {}
    for k, (_, s, e) in enumerate(blocks):
        ins = []
        for i in range(s + 1, e):
            t = L[i].split(';')[0].strip()
            if t and not t.startswith('.'):
                ins.append((i, t))
        insts[k] = ins
        fall = True
        for _, t in ins:
            op = t.split()[0]
            if op.startswith('s_cbranch'):
                succ[k].append(idx[t.split()[1]])
            elif op == 's_branch':
                succ[k].append(idx[t.split()[1]])
                fall = False
            elif op in ('s_endpgm', 's_setpc_b64'):
                fall = False
        if fall and k + 1 < len(blocks):
            succ[k].append(k + 1)
    preds = defaultdict(list)
    for k, ss in succ.items():
        for s in ss:
            preds[s].append(k)
    return blocks, insts, preds


def slot_w(t):
    m = re.match(r'v_writelane_b32 (v\d+), (s\d+|vcc_lo|vcc_hi|m0|exec_lo|exec_hi), (\d+)$', t)
    return ((m.group(1), int(m.group(3))), m.group(2)) if m else None


def slot_r(t):
    m = re.match(r'v_readlane_b32 (s\d+|vcc_lo|vcc_hi|m0), (v\d+), (\d+)$', t)
    return ((m.group(2), int(m.group(3))), m.group(1)) if m else None


def vregs(tok):
    m = re.fullmatch(r'v(\d+)', tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r'v\[(\d+):(\d+)\]', tok)
    return set(range(int(m.group(1)), int(m.group(2)) + 1)) if m else set()


def main():
    L = extract(sys.argv[1], sys.argv[2])
    show_all = '--all' in sys.argv
    blocks, insts, preds = cfg(L)
    spill = sorted({int(slot_w(t)[0][0][1:]) for k in insts for _, t in insts[k] if slot_w(t)})
    print(f"{len(L)} lines; spill VGPRs: {spill}")
    # other writes to the spill VGPRs
    clobbers = []
    for k in insts:
        for i, t in insts[k]:
            p = t.split(None, 1)
            if len(p) < 2 or p[0] == 'v_writelane_b32':
                continue
            if p[0].startswith(('global_store', 'buffer_store', 'ds_write', 'ds_store', 'flat_store',
                                'scratch_store', 's_', 'v_readlane', 'v_readfirstlane', 'v_cmp')):
                continue
            if vregs(p[1].split(',')[0].strip()) & set(spill):
                clobbers.append((i + 1, t))
    print(f"other writes to spill VGPRs: {len(clobbers)}")
    for c in clobbers[:20]:
        print("   ", c)
    # reaching definitions per slot
    out = {k: {} for k in range(len(blocks))}
    changed = True
    while changed:
        changed = False
        for k in range(len(blocks)):
            d = defaultdict(set)
            for p in preds[k]:
                for s, v in out[p].items():
                    d[s] |= v
            for i, t in insts[k]:
                w = slot_w(t)
                if w:
                    d[w[0]] = {i}
            d = dict(d)
            if d != out[k]:
                out[k] = d
                changed = True
    nread = nmulti = nundef = 0
    for k in range(len(blocks)):
        d = defaultdict(set)
        for p in preds[k]:
            for s, v in out[p].items():
                d[s] |= v
        for i, t in insts[k]:
            r = slot_r(t)
            if r and int(r[0][0][1:]) in spill:
                nread += 1
                ws = sorted(w + 1 for w in d.get(r[0], set()))
                nmulti += len(ws) > 1
                nundef += len(ws) == 0
                if show_all or len(ws) != 1:
                    print(f"   read line {i + 1} {r[0]} -> {r[1]}: written at {ws}")
            w = slot_w(t)
            if w:
                d[w[0]] = {i}
    print(f"spill-lane reads: {nread}; reached by no write: {nundef}; by several writes: {nmulti}")
    # per loop
    stats, hdr = defaultdict(Counter), None
    for l in L:
        if re.match(r'^(\.LBB|; %bb)', l):
            m = re.search(r'Header=(\S+) Depth=(\d+)', l)
            m2 = re.search(r'Loop Header: Depth=(\d+)', l)
            hdr = (m.group(1), int(m.group(2))) if m else (
                (l.split(':')[0].lstrip('.').lstrip('L'), int(m2.group(1))) if m2 else None)
            continue
        t = l.split(';')[0].strip()
        if not t or t.startswith('.'):
            continue
        op = t.split()[0]
        st = stats[hdr]
        st['instructions'] += 1
        st['valu'] += op.startswith('v_')
        r = slot_r(t)
        st['readlane_spill'] += bool(r) and int(r[0][0][1:]) in spill
        st['writelane_spill'] += bool(slot_w(t))
    for h, v in stats.items():
        print("loop" if h else "outside loops", h or "", dict(v))


if __name__ == '__main__':
    main()
