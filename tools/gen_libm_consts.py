"""Read the constants of the host C library's logf / expf (the FMA variants its IFUNC
resolvers select on this CPU) out of libm, and check them against semtsdf_libm.h.

The reference's association runs on the host (src/SfM_CUDA/tsdf.cu:318,329,343) with the
platform's logf/expf; slam-maskrcnn_amd/csrc/semtsdf_libm.h restates glibc's algorithm with
these constants so the device reproduces those f32 values.  Method: `nm -D` gives the IFUNC
resolver of logf/expf; the resolver's `cmovne` target is the FMA variant; the RIP-relative
operands of that function (objdump's `# addr` comments) are its tables and coefficients.
Usage: python tools/gen_libm_consts.py [path/to/libm.so.6]
"""
import re
import struct
import subprocess
import sys
import os

LIBM = sys.argv[1] if len(sys.argv) > 1 else "/lib/x86_64-linux-gnu/libm.so.6"
HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "slam-maskrcnn_amd", "csrc",
                   "semtsdf_libm.h")


def dis(start, n=60):
    out = subprocess.run(["objdump", "-d", "--no-show-raw-insn", f"--start-address={start:#x}",
                          f"--stop-address={start + 4 * n:#x}", LIBM], capture_output=True, text=True).stdout
    return [ln for ln in out.splitlines() if re.match(r"\s+[0-9a-f]+:", ln)]


def ifunc(sym):
    for ln in subprocess.run(["nm", "-D", LIBM], capture_output=True, text=True).stdout.splitlines():
        f = ln.split()
        if len(f) == 3 and f[1] == "i" and f[2].startswith(sym + "@@"):
            return int(f[0], 16)
    raise SystemExit(f"no IFUNC {sym} in {LIBM}")


def fma_variant(sym):
    lines = dis(ifunc(sym), 12)
    lea = [int(re.search(r"# ([0-9a-f]+)", ln).group(1), 16) for ln in lines if "lea" in ln and "#" in ln]
    assert any("cmovne" in ln for ln in lines), lines
    return lea[-1]  # the candidate moved in by cmovne (FMA + AVX2 usable)


def operands(fn):
    addrs = []
    for ln in dis(fn, 40):
        m = re.search(r"# ([0-9a-f]+)", ln)
        if m:
            addrs.append((int(m.group(1), 16), ln.split("\t")[-1]))
        if ln.strip().endswith("ret"):
            break
    return addrs


def main():
    data = open(LIBM, "rb").read()
    d = lambda a: struct.unpack("<d", data[a:a + 8])[0]
    q = lambda a: struct.unpack("<Q", data[a:a + 8])[0]
    lg = operands(fma_variant("logf"))
    tab = [a for a, ins in lg if ins.startswith("lea")][0]
    coef = sorted({a for a, ins in lg if not ins.startswith("lea") and a > tab})
    logf_tab = [(d(tab + 16 * i), d(tab + 16 * i + 8)) for i in range(16)]
    ln2, a0, a1, a2 = (d(a) for a in coef[:4])
    ex = operands(fma_variant("expf"))
    etab = [a for a, ins in ex if ins.startswith("lea")][0]
    ec = sorted({a for a, ins in ex if not ins.startswith("lea") and a > etab})
    shift, invln2n, c0, c1, c2 = (d(a) for a in ec[:5])
    expf_tab = [q(etab + 8 * i) for i in range(32)]
    hdr = open(HDR).read()
    want = [f"{{{x.hex()}, {y.hex()}}}" for x, y in logf_tab] + [f"0x{v:016x}ull" for v in expf_tab]
    want += [f"kLogfLn2 = {ln2.hex()}", f"kLogfA0 = {a0.hex()}", f"kLogfA1 = {a1.hex()}", f"kLogfA2 = {a2.hex()}",
             f"kExpfShift = {shift.hex()}", f"kExpfInvLn2N = {invln2n.hex()}", f"kExpfC0 = {c0.hex()}",
             f"kExpfC1 = {c1.hex()}", f"kExpfC2 = {c2.hex()}"]
    norm = lambda s: s.replace("0x1.0000000000000p+0", "0x1.0p+0").replace("0x1.8000000000000p+52", "0x1.8p+52")
    hnorm = norm(re.sub(r"\s+", " ", hdr))
    missing = [w for w in want if norm(w) not in hnorm]
    for w in want:
        print(w)
    if missing:
        raise SystemExit(f"{len(missing)} constants differ from {HDR}: {missing[:4]}")
    print(f"all {len(want)} constants of {LIBM} match {os.path.basename(HDR)}")


if __name__ == "__main__":
    main()
