"""List every s_barrier in libsesa's gfx950 code that a wave can reach with its own LDS operations still in flight.

Round 6 (BS-Roformer cross-stream discrepancy): the compiler drops the `s_waitcnt lgkmcnt(0)` of a __syncthreads()
whose workgroup fence it can prove needs no cross-address-space ordering -- LLVM's memory model takes LDS operations of
all waves to execute in one global order.  This is a dataflow over each kernel's basic blocks: a block's state is
"an LDS write (or read) issued and not yet waited for", joined over predecessors (loop back edges included), cleared by
an s_waitcnt whose lgkmcnt is 0, and every s_barrier reached in that state is reported.

  python tools/barrier_scan.py [libsesa.so] [--reads]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_guard import LLVM, device_images  # noqa: E402

FN = re.compile(r"^([0-9a-f]+) <(.+)>:$")
INS = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):[^<]*(?:<([^>]+)>)?\s*$")


def lds_kind(op):
    if not op.startswith("ds_"):
        return None
    if op.startswith(("ds_read", "ds_load")):
        return "r"
    if op in ("ds_swizzle_b32", "ds_bpermute_b32", "ds_permute_b32") or op.startswith("ds_nop"):
        return None
    return "w"


def clears(op, args):
    if op != "s_waitcnt":
        return False
    m = re.search(r"lgkmcnt\((\d+)\)", args)
    return (m is not None and m.group(1) == "0") or args.strip() in ("0", "0x0")


def functions(asm):
    """(name, [(addr, op, args, branch_target_addr or None)])"""
    fn, base, body = None, 0, []
    for line in asm.splitlines():
        m = FN.match(line)
        if m:
            if fn:
                yield fn, body
            fn, base, body = m.group(2), int(m.group(1), 16), []
            continue
        m = INS.match(line) if fn else None
        if not m:
            continue
        tgt = None
        if m.group(4) and (m.group(1).startswith("s_cbranch") or m.group(1) == "s_branch"):
            o = re.search(r"\+0x([0-9a-f]+)$", m.group(4))
            tgt = base + (int(o.group(1), 16) if o else 0)
        body.append((int(m.group(3), 16), m.group(1), m.group(2), tgt))
    if fn:
        yield fn, body


def scan_fn(body, want):
    """Barrier addresses reachable with an outstanding LDS op of a kind in `want`."""
    at = {a: i for i, (a, _, _, _) in enumerate(body)}
    leaders = {0}
    for i, (a, op, args, tgt) in enumerate(body):
        if op.startswith("s_cbranch") or op == "s_branch" or op == "s_endpgm":
            leaders.add(i + 1)
        if tgt is not None and tgt in at:
            leaders.add(at[tgt])
    starts = sorted(x for x in leaders if x < len(body))
    blocks = [(s, starts[k + 1] if k + 1 < len(starts) else len(body)) for k, s in enumerate(starts)]
    bidx = {s: k for k, (s, e) in enumerate(blocks)}
    succ = {}
    for k, (s, e) in enumerate(blocks):
        a, op, args, tgt = body[e - 1]
        out = []
        if tgt is not None and tgt in at:
            out.append(bidx[at[tgt]])
        if op == "s_endpgm" or op == "s_branch":
            pass
        elif k + 1 < len(blocks):
            out.append(k + 1)
        succ[k] = out
    state_in = {k: False for k in range(len(blocks))}
    hits = set()
    changed = True
    while changed:
        changed = False
        for k, (s, e) in enumerate(blocks):
            st = state_in[k]
            for i in range(s, e):
                a, op, args, _ = body[i]
                if clears(op, args):
                    st = False
                elif op == "s_barrier" and st:
                    hits.add(a)
                if lds_kind(op) in want:
                    st = True
            for o in succ[k]:
                if st and not state_in[o]:
                    state_in[o] = True
                    changed = True
    return sorted(hits)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    want = {"w", "r"} if "--reads" in sys.argv else {"w"}
    so = args[0] if args else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                           "sesa-audio-separation_amd", "sesa", "_native", "libsesa.so")
    total = 0
    with tempfile.TemporaryDirectory() as td:
        for n, img in enumerate(device_images(so)):
            f = os.path.join(td, f"co{n}.o")
            open(f, "wb").write(img)
            asm = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", "--no-show-raw-insn", f],
                                 capture_output=True, text=True, check=True).stdout
            for fn, body in functions(asm):
                hits = scan_fn(body, want)
                if hits:
                    total += len(hits)
                    print(f"{len(hits):3d} barrier(s) with LDS ops in flight: {fn}")
    print(f"barrier_scan: {total} s_barrier sites reachable with un-waited LDS {'ops' if len(want) > 1 else 'writes'}")
    return total


if __name__ == "__main__":
    sys.exit(1 if main() else 0)
