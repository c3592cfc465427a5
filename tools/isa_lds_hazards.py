"""Scan gfx950 assembly for reads of a VGPR that an in-flight LDS read is still filling.

Hand-written inline asm (attention.hip frag_tr_asm, the lse / D reads; gemm_pp3.h cnt_bias)
issues several ds_read instructions and waits for them itself, so hipcc's waitcnt pass does
not protect their destinations.  Two ways that goes wrong, both found in round 3's shipped
kernels and both timing-dependent (an LDS read can return before the wave issues its next
instruction when the LDS queue is backed up):
  * address clobber: a later ds_read in the same asm takes its address from a register an
    earlier ds_read of the asm is filling (asm outputs without "&" early-clobber);
  * stale read: a VALU / MFMA instruction reads such a destination before the s_waitcnt
    lgkmcnt that retires it (hipcc copying an asm output it believes is already final).
Usage: python tools/isa_lds_hazards.py file.s [...]  -> one line per kernel with hazards;
exit status 1 if any.  (tests/test_isa_cpu.py runs it over the device assembly of the
kernels that use such asm.)
"""
import re
import sys

_KERNEL = re.compile(r"^(_Z\S+):")
_LGKM_DEST = re.compile(r"^(ds_read\w*|ds_bpermute\w*|ds_permute\w*|ds_swizzle\w*)\s")


def _regs(text):
    out = set()
    for bank, a, b in re.findall(r"([va])\[(\d+):(\d+)\]", text):
        out.update((bank, r) for r in range(int(a), int(b) + 1))
    for bank, x in re.findall(r"(?<![\[:\w])([va])(\d+)", text):
        out.add((bank, int(x)))
    return out


def scan(lines):
    """{kernel: [(line_no, kind, text)]}: an instruction reading a register that an LDS read
    still in flight (not yet retired by an s_waitcnt lgkmcnt) is filling.  LGKM operations
    retire in order (the scan models lgkmcnt(N) as "all but the N youngest"); a scalar load
    in flight makes any lgkmcnt wait but (0) unreliable, so those reset nothing."""
    hits, kernel, fifo = {}, None, []
    smem = False
    for no, raw in enumerate(lines, 1):
        m = _KERNEL.match(raw)
        if m:
            kernel, fifo, smem = m.group(1), [], False
            continue
        t = raw.split(";")[0].strip()
        if not t or kernel is None or t.startswith("."):
            if t.startswith(".LBB"):
                fifo, smem = [], False  # straight-line sequences only (no cross-block state)
            continue
        if t.startswith("s_branch") or t.startswith("s_cbranch") or t.startswith("s_setpc"):
            fifo, smem = [], False
            continue
        w = re.match(r"s_waitcnt.*lgkmcnt\((\d+)\)", t)
        if w:
            n = int(w.group(1))
            if n == 0:
                fifo, smem = [], False
            elif not smem:
                fifo = fifo[len(fifo) - n:] if n < len(fifo) else fifo
            continue
        op, _, args = t.partition(" ")
        if op.startswith("s_load") or op.startswith("s_buffer_load"):
            smem = True
            continue
        pend = set().union(*fifo) if fifo else set()
        if not (op.startswith("ds_") or op.startswith("v_") or op.startswith("buffer_") or op.startswith("global_")):
            continue
        parts = [x.strip() for x in args.split(",")]
        stores = op.startswith("ds_write") or "store" in op
        srcs = _regs(",".join(parts if stores else parts[1:]))
        if pend and srcs & pend:
            kind = "address clobber" if op.startswith("ds_") else "stale read"
            hits.setdefault(kernel, []).append((no, kind, t))
        if op.startswith("ds_"):
            fifo.append(_regs(parts[0]) if _LGKM_DEST.match(t) else set())
    return hits


def main(paths):
    bad = 0
    for p in paths:
        with open(p) as f:
            hits = scan(f.read().split("\n"))
        for k, v in hits.items():
            bad += len(v)
            print(f"{p}: {k[:80]}: {len(v)} ({', '.join(sorted({x[1] for x in v}))}); first at line {v[0][0]}: {v[0][2]}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
