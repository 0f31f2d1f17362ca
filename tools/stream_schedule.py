"""CPU model of the streaming kernel's LDS ring schedule (csrc/mha_hd64_stream.hip), with a
race check ("prove the 8-wave ring schedule race-free, or fix it").

The kernel's control flow is wave-uniform: every wave of a workgroup runs the same sequence of
LDS-DMA issues, counted `s_waitcnt vmcnt(N)` waits, `s_barrier`s and LDS reads; only the timing
differs between waves. So one op sequence describes every wave, and a schedule is race-free for
EVERY timing when, in that sequence:

  RAW  every LDS read of ring slot S holding global tile T comes after a barrier that comes after
       a wait (in program order) that covers every DMA piece of T (each wave DMAs its own pieces
       of every tile, so the covering wait must be the issuing wave's, followed by a barrier
       before any wave reads);
  WAR  every DMA into slot S (a newer tile) comes after a barrier that comes after every read of
       the tile the slot held before (a fast wave's refill may not overtake a slow wave's read;
       a read returns the bytes at issue, so a read issued before the DMA needs no more);
  OWN  reads of a wave's own Q rows come after a wait covering that wave's Q DMA (no barrier:
       each wave DMAs and reads its own 32 rows);
  ZERO the zeroed V image ("tile -1") is written by ds_write, drained (lgkmcnt), then a barrier,
       before any wave reads it.

`s_waitcnt vmcnt(N)` = all but the wave's N youngest vector-memory ops are done; LDS-DMA pieces,
buffer stores and Q pieces count together in issue order (MI355X_MICROARCH.md, vmcnt).

The op sequence below restates the kernel (line references to mha_hd64_stream.hip):
  prologue           :347-366 (issue_q, L0 tiles, zero the V image of slot kSM, wait, barrier,
                      tiles L0..L-1), :662-683 (read_q, K of tile 0, wait, barrier)
  loop top           :690-692 (lgkmcnt(0), issue_q(nxt))
  step (all kinds)   :458-646 (phase A: K reads of tile g+1, V reads of tile g-1, the refill DMA of
                      tile g+L; FIRST: the previous item's epilogue stores after the refill; the
                      step's wait and barrier by NW and kind)
  before LAST        :725-726 (NW 8 two-tile items: vmcnt(0); read_q)
  flush              :749-763 (V reads of the last tile, epilogue stores, vmcnt(0))

    python tools/stream_schedule.py            # check both forms over a sweep of item sequences
"""
import itertools
import sys


def ring_params(nw):
    slots = 8 if nw == 8 else 4
    lead = 4 if nw == 8 else 2
    kpw = 8 // nw  # DMA pieces per wave per image (K or V) of a tile
    return slots, lead, 2 * kpw


def kernel_ops(nw, items_nt, out_f32=False, mutate=None):
    """Op sequence of one wave for a workgroup whose items have the given (even) tile counts.

    Ops: ('dma', tile, slot) one LDS-DMA piece; ('qdma', item) one Q piece; ('store',) one output
    store; ('wait', n) vmcnt(n); ('bar',); ('read', kind, tile, slot) kind 'K' / 'V';
    ('readq', item); ('zero', slot) ds_write of the zero V image; ('lgkm',) lgkmcnt(0)."""
    slots, lead, kpiece = ring_params(nw)
    # mutations (tests/test_stream_schedule.py: the checker must flag each of them)
    if mutate == "lead+2":  # refill two tiles further ahead in the same ring
        lead += 2
    odd_wait = 2 * kpiece if mutate == "odd_wait_loose" else kpiece
    nstores = 8 if out_f32 else 4
    ops = []
    nload = [0]  # the loader cursor's global tile (the kernel's ld / ld_advance)

    def issue_tile():
        t = nload[0]
        for _ in range(kpiece):
            ops.append(("dma", t, t % slots))
        nload[0] += 1

    def issue_q(item):
        for _ in range(4):
            ops.append(("qdma", item))

    # ---- kernel prologue (:347-366) ----
    l0 = 2 if nw == 8 else lead
    issue_q(0)
    for _ in range(l0):
        issue_tile()
    ops.append(("zero", slots - 1))
    ops.append(("wait", (l0 - 1) * kpiece))
    if mutate != "no_prologue_barrier":
        ops.append(("bar",))
    for _ in range(l0, lead):
        issue_tile()
    # first item's Q fragments and tile 0's QK^T (:662-680); the reads are consumed there
    ops.append(("readq", 0))
    ops.append(("read", "K", 0, 0))
    ops.append(("lgkm",))  # (the MFMAs consume the reads: LDS ops done, in order)
    ops.append(("wait", (lead - 2) * kpiece))
    ops.append(("bar",))

    gb = 0
    prev = False
    nitems = len(items_nt)
    for i, nt in enumerate(items_nt):
        assert nt >= 2 and nt % 2 == 0
        # loop top (:690-692): the next item's Q (an empty descriptor past the last item)
        ops.append(("lgkm",))
        issue_q(i + 1 if i + 1 < nitems else None)
        # steps t = 0 .. nt-1: FIRST, middle / tail pairs, LAST (:697-728)
        for t in range(nt):
            g = gb + t
            first, last = t == 0, t == nt - 1
            if last:
                if nw == 8 and nt == 2 and mutate != "no_two_tile_wait":
                    ops.append(("wait", 0))
                ops.append(("readq", i + 1 if i + 1 < nitems else None))
            # phase A (:557-581): K of tile g + 1 (reads at s = 0..3), V of tile g - 1 (s = 1, 2),
            # the refill pieces dma(s) for s < kpiece, interleaved in that order
            ops.append(("read", "K", g + 1, (g + 1) % slots))
            ops.append(("read", "K", g + 1, (g + 1) % slots))
            for s in range(4):
                if s < 2:
                    ops.append(("read", "K", g + 1, (g + 1) % slots))
                if s in (1, 2):
                    ops.append(("read", "V", g - 1, (g - 1) % slots))
                if s < kpiece:
                    t_ = nload[0]
                    ops.append(("dma", t_, t_ % slots))
            nload[0] += 1
            ops.append(("lgkm",))  # phase B's MFMAs consume the K / V fragments
            if first and prev:
                for _ in range(nstores):
                    ops.append(("store",))
            # the step's wait and barrier (:627-643)
            if nw == 4:
                ops.append(("wait", kpiece if mutate == "nw4_wait_loose" else 0))
                ops.append(("bar",))
            elif (t % 4 == 3) if mutate == "every_4th_barrier" else (t % 2 == 1):  # odd t (items start on even tiles)
                ops.append(("wait", odd_wait))
                ops.append(("bar",))
            elif first and not prev:
                ops.append(("wait", 2 * kpiece + 4 + (kpiece if mutate == "first_wait_loose" else 0)))
                ops.append(("bar",))
        prev = True
        gb += nt
    # flush (:749-763): the last item's last tile
    e = gb - 1
    ops.append(("read", "V", e, e % slots))
    ops.append(("read", "V", e, e % slots))
    ops.append(("lgkm",))
    for _ in range(nstores):
        ops.append(("store",))
    ops.append(("wait", 0))
    return ops


def check(ops, nw):
    """Violations of RAW / WAR / OWN / ZERO (see the module docstring) as strings."""
    slots, _, _ = ring_params(nw)
    vm = []  # positions of vm ops in issue order
    covered_at = {}  # vm op index -> position of the first wait that covers it
    for p, op in enumerate(ops):
        if op[0] in ("dma", "qdma", "store"):
            vm.append(p)
        elif op[0] == "wait":
            n = op[1]
            for idx in range(0, max(0, len(vm) - n)):
                covered_at.setdefault(idx, p)
    pos_vm = {p: i for i, p in enumerate(vm)}
    bars = [p for p, op in enumerate(ops) if op[0] == "bar"]

    def bar_between(a, b):
        return any(a < x < b for x in bars)

    errors = []
    # the DMA pieces of each tile, and who holds each slot when
    pieces = {}
    for p, op in enumerate(ops):
        if op[0] == "dma":
            pieces.setdefault(op[1], []).append(p)
    qpieces = {}
    for p, op in enumerate(ops):
        if op[0] == "qdma":
            qpieces.setdefault(op[1], []).append(p)
    for p, op in enumerate(ops):
        if op[0] == "read":
            _, kind, tile, slot = op
            if tile < 0:  # the zeroed V image
                z = [q for q, o in enumerate(ops) if o[0] == "zero" and o[1] == slot]
                ok = any(any(o[0] == "lgkm" and zq < x < p for x, o in enumerate(ops)) and
                         any(zq < b < p and any(o[0] == "lgkm" and zq < x < b for x, o in enumerate(ops)) for b in bars)
                         for zq in z)
                if not ok:
                    errors.append(f"ZERO: read of the zero image at {p} not behind drained writes + barrier")
                # and no DMA into that slot before the read
                if any(o[0] == "dma" and o[2] == slot and q < p for q, o in enumerate(ops)):
                    errors.append(f"ZERO: slot {slot} refilled before its zero image is read at {p}")
                continue
            ps = pieces.get(tile)
            if not ps:
                errors.append(f"RAW: read of tile {tile} at {p}: never issued")
                continue
            for d in ps:
                w = covered_at.get(pos_vm[d])
                if w is None or not (w < p and bar_between(w, p)):
                    errors.append(f"RAW: {kind} read of tile {tile} (slot {slot}) at {p}: piece at {d} "
                                  f"not waited ({w}) + barrier before it")
                    break
            # the slot still holds this tile: no newer tile's DMA into it issued before the read
            newer = [q for q, o in enumerate(ops) if o[0] == "dma" and o[2] == slot and o[1] > tile and q < p]
            if newer:
                errors.append(f"WAR: {kind} read of tile {tile} at {p} after a newer tile's DMA into slot {slot} at {newer[0]}")
        elif op[0] == "dma":
            _, tile, slot = op
            # every read of an older tile in this slot needs a barrier between it and this DMA
            for q in range(p):
                o = ops[q]
                if o[0] == "read" and o[3] == slot and o[2] < tile and not bar_between(q, p):
                    errors.append(f"WAR: DMA of tile {tile} into slot {slot} at {p} not behind a barrier after "
                                  f"the {o[1]} read of tile {o[2]} at {q}")
                    break
            # and none of those reads comes after it (an old tile read later: the slot was reused early)
            for q in range(p + 1, len(ops)):
                o = ops[q]
                if o[0] == "read" and o[3] == slot and 0 <= o[2] < tile:
                    errors.append(f"WAR: {o[1]} read of tile {o[2]} at {q} after the DMA of tile {tile} into "
                                  f"slot {slot} at {p}")
                    break
        elif op[0] == "readq":
            ps = qpieces.get(op[1], [])
            for d in ps:
                w = covered_at.get(pos_vm[d])
                if w is None or w > p:
                    errors.append(f"OWN: Q read of item {op[1]} at {p} before its DMA at {d} is waited")
                    break
            # the region is not refilled (next item's Q) before this read: issue_q comes after
            later_q = [d for it, dl in qpieces.items() if it != op[1] for d in dl if d < p and
                       (not qpieces.get(op[1]) or d > max(qpieces[op[1]]))]
            if later_q:
                errors.append(f"OWN: Q region refilled at {later_q[0]} before the read of item {op[1]} at {p}")
    # every vm op is waited before the end (the grid drains)
    if vm and covered_at.get(len(vm) - 1) is None:
        errors.append("drain: vector-memory ops still in flight at exit")
    return errors


# (mutation, the form it applies to): each must be flagged. Barriers on even steps instead of odd
# ones would be race-free too: a slot is reused 3 (NW 4: 1) steps after its last read and a refill
# is read 3 (1) steps after issue, so any barrier every second step separates both.
MUTATIONS = (("lead+2", 4), ("lead+2", 8), ("odd_wait_loose", 8), ("every_4th_barrier", 8),
             ("no_prologue_barrier", 4), ("no_prologue_barrier", 8), ("no_two_tile_wait", 8),
             ("first_wait_loose", 8), ("nw4_wait_loose", 4))


def sweep(nws=(4, 8), max_items=3, tiles=(2, 4, 6, 8, 16, 34), mutate=None):
    """Check every item sequence of 1..max_items items drawn from `tiles` (even tile counts: one-
    and two-tile calls give 2, 1024 keys 16, 2048 keys 32 + ...), both output types."""
    n = 0
    bad = []
    for nw in nws:
        for k in range(1, max_items + 1):
            for seq in itertools.product(tiles, repeat=k):
                for f32 in (False, True):
                    errs = check(kernel_ops(nw, list(seq), f32, mutate), nw)
                    n += 1
                    if errs:
                        bad.append((nw, seq, f32, errs[:3]))
    return n, bad


if __name__ == "__main__":
    n, bad = sweep()
    for b in bad[:20]:
        print(b)
    print(f"checked {n} item sequences; {len(bad)} with violations")
    sys.exit(1 if bad else 0)
