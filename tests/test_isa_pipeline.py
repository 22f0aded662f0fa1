"""The integrate's software pipeline survives compilation ("Stages, software-pipelined").

The project stage of unit k+1 issues its pixel gathers before the compute stage of unit k, which
waits only for unit k's state loads: in the machine code the first `s_waitcnt vmcnt(N)` after a
run of gathers keeps N > 0 (the gathers stay in flight).  The compiler falls back to vmcnt(0)
when it cannot order the pending vector-memory operations -- for instance after FLAT atomics or
stores through a pointer it cannot place in the global address space (a pointer loaded from
memory is generic) -- and the gathers' latency then lands on every group: r05 lost ~3.5 us per
512^3 frame that way until the rare-path pointers were cast to the global address space.  This
test disassembles the built library's gfx950 code object (no GPU needed) and checks the kernels
the bench runs: no FLAT memory instructions, and no vmcnt(0) right after a run of gathers.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "slam-maskrcnn_amd", "semtsdf", "libsemtsdf.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

# k_integrate<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN> of the bench lines: C3, C4 shard, C2
KERNELS = {
    "C3": "_ZN7semtsdf11k_integrateILb1ELb1ELb0ELb0ELb0ELb0ELb1EEEvNS_13IntegrateArgsENS_8UnitGridEj",
    "C4 shard": "_ZN7semtsdf11k_integrateILb1ELb1ELb0ELb0ELb0ELb1ELb1EEEvNS_13IntegrateArgsENS_8UnitGridEj",
    "C2": "_ZN7semtsdf11k_integrateILb0ELb0ELb0ELb0ELb0ELb0ELb1EEEvNS_13IntegrateArgsENS_8UnitGridEj",
}
GATHER = re.compile(r"^\s*global_load_dword(x2)?\s")


def _disassemble(tmp_path):
    lib = tmp_path / "libsemtsdf.so"
    shutil.copy(LIB, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, capture_output=True, cwd=tmp_path, timeout=120)
    co = [p for p in tmp_path.iterdir() if p.name.endswith("gfx950")]
    assert co, "no gfx950 code object in the library"
    out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", str(co[0])], check=True, capture_output=True,
                         text=True, timeout=300).stdout
    return out


def _function(dis, name):
    m = re.search(r"^[0-9a-f]+ <" + re.escape(name) + r">:\n", dis, re.M)
    assert m, name
    end = re.search(r"^[0-9a-f]+ <\w+>:\n", dis[m.end():], re.M)
    return dis[m.end():m.end() + end.start()] if end else dis[m.end():]


def _loop_ranges(body, fstart):
    """[target, branch] address ranges of the backward branches (the loops) of one function."""
    ranges = []
    for line in body:
        m = re.search(r"s_(?:c)?branch\w*\s.*//\s*([0-9A-F]+):.*<\w+\+0x([0-9a-f]+)>", line)
        if m:
            at, tgt = int(m.group(1), 16), fstart + int(m.group(2), 16)
            if tgt < at:
                ranges.append((tgt, at))
    return ranges


def _addr(line):
    m = re.search(r"//\s*([0-9A-F]+):", line)
    return int(m.group(1), 16) if m else None


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_integrate_gathers_stay_in_flight(tmp_path):
    dis = _disassemble(tmp_path)
    for cfg, name in KERNELS.items():
        fstart = int(re.search(r"^([0-9a-f]+) <" + re.escape(name) + r">:", dis, re.M).group(1), 16)
        body = _function(dis, name).splitlines()
        flat = [l for l in body if re.match(r"^\s*flat_", l)]
        assert not flat, (cfg, flat[:3])
        loops = _loop_ranges(body, fstart)
        waits, k = [], 0
        while k < len(body):
            if GATHER.match(body[k]):
                run, m = [k], k + 1
                while m < len(body) and m - run[-1] <= 3:
                    if GATHER.match(body[m]):
                        run.append(m)
                    m += 1
                at = _addr(body[run[-1]])
                # runs of gathers inside a loop (the steady state of a list; the primes before
                # the loops classify right after their gathers and wait for them legitimately)
                if len(run) >= 4 and any(lo <= at <= hi for lo, hi in loops):
                    for n in range(run[-1] + 1, min(run[-1] + 40, len(body))):
                        w = re.search(r"s_waitcnt\s.*vmcnt\((\d+)\)", body[n])
                        if w:
                            waits.append(int(w.group(1)))
                            break
                k = m
            else:
                k += 1
        assert len(waits) >= 1, (cfg, waits)  # at least one list's steady loop
        assert min(waits) > 0, (cfg, waits)
