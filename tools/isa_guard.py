"""Build guard: fail if libsesa's gfx950 code contains a packed-fp32 VALU instruction with a source op_sel.

Round 6 finding (profiles/r06_pk_opsel_hazard.txt): on MI355X, v_pk_add_f32 / v_pk_mul_f32 (/ fma) whose
op_sel picks the high half of a source for the low result -- the form the SLP vectorizer emits for complex
arithmetic -- return wrong values while another wave on the same CU is executing MFMAs (tools/victim_stress.py
form2 / form3: 4-6 of 40 chained runs corrupted; the same chain without op_sel, 0 of 40).  That was the cross-stream
discrepancy of rounds 4-5: the FFT kernels (STFT / iSTFT) computed wrong columns whenever another stream's MFMA
kernel shared their CUs.  libsesa is built with -fno-slp-vectorize and no hand-written packed op uses op_sel; this
check keeps it that way.

  python tools/isa_guard.py path/to/libsesa.so      (exit 1 and a listing if any such instruction is present)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
BAD = re.compile(r"\bv_pk_(add|mul|fma)_f32\b[^\n]*\bop_sel:\[")


def device_images(so_path):
    """The gfx950 code objects of every offload bundle in the library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fatbin")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", so_path,
                               os.path.join(td, "stripped")])
        data = open(fat, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(MAGIC))[0]
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 1)
    return out


def scan(so_path):
    hits = []
    images = device_images(so_path)
    with tempfile.TemporaryDirectory() as td:
        for i, img in enumerate(images):
            f = os.path.join(td, f"co{i}.o")
            open(f, "wb").write(img)
            asm = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", "--no-show-raw-insn", f],
                                 capture_output=True, text=True, check=True).stdout
            fn = None
            for line in asm.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if m:
                    fn = m.group(1)
                elif BAD.search(line):
                    hits.append((fn, line.strip()))
    return len(images), hits


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                            "sesa-audio-separation_amd", "sesa", "_native", "libsesa.so")
    n, hits = scan(so)
    if not n:
        print(f"isa_guard: no gfx950 code objects found in {so}", file=sys.stderr)
        sys.exit(1)
    if hits:
        kernels = sorted({h[0] for h in hits})
        print(f"isa_guard: {len(hits)} packed-fp32 instructions with a source op_sel in {len(kernels)} kernels of {so} "
              f"(unsafe beside MFMA work on gfx950; see tools/isa_guard.py):", file=sys.stderr)
        for k in kernels[:20]:
            print(f"   {k}: e.g. {next(h[1] for h in hits if h[0] == k)}", file=sys.stderr)
        sys.exit(1)
    print(f"isa_guard: {so}: {n} gfx950 code objects, no packed-fp32 op_sel instruction")


if __name__ == "__main__":
    main()
