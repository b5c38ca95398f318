"""The release tiled kernels keep their round pipeline (CPU test: hipcc
cross-compiles the kernels to gfx950 assembly, nothing runs).

Each tiled kernel keeps DEPTH - 1 rounds of loads in flight while it
processes one.  The wait for a round's data -- the
`s_waitcnt vmcnt(N)` right before the permlane transpose that starts
processing it -- must leave at least one further round (4 loads)
outstanding.  Round 2 found the compute gather kernel waiting vmcnt(1) /
vmcnt(0) at its loop head instead (a noreturn trap in its slot wait had
reshaped the CFG), i.e. no prefetch across rounds; this test keeps that
from coming back unnoticed in any product kernel."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hadoofus_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
MIN_OUTSTANDING = 4  # one round of data loads


@pytest.fixture(scope="module")
def release_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm") / "kernels.s"
    # the release build's device flags (hadoofus_amd/build.py), device code only
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                           "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "-I" + os.path.join(ROOT, "include"),
                           "-I" + CSRC, "-o", str(out), os.path.join(CSRC, "crc32c_kernels.hip")],
                          stderr=subprocess.DEVNULL)
    return out.read_text().splitlines()


def round_waits(lines):
    """{tiled kernel symbol: [N of every vmcnt(N) wait that precedes the first
    use of a round's data]}: the permlane transpose, or in the verify +
    copy-out kernels of aligned data the copy-out's 1 KiB stores of the
    loaded registers, which come first."""
    name, res, kernels = None, {}, set()
    for i, line in enumerate(lines):
        m = re.match(r"^(_ZN11hdfs_crc32c\w*crc32c_tiles_kernel\w+):", line)
        if m:
            name = m.group(1)
            kernels.add(name)
            continue
        if re.match(r"^_ZN\w+:", line):
            name = None
        m = re.search(r"s_waitcnt vmcnt\((\d+)\)", line)
        if m and name:
            nxt = [x for x in lines[i + 1:i + 12] if x.strip() and not x.strip().startswith(";")][:6]
            if any("v_permlane16_swap" in x or "buffer_store_dwordx4" in x for x in nxt):
                res.setdefault(name, []).append(int(m.group(1)))
    return kernels, res


def test_release_tiled_kernels_keep_rounds_in_flight(release_asm):
    kernels, waits = round_waits(release_asm)
    assert kernels, "no tiled kernels in the release build"
    assert set(waits) == kernels, sorted(kernels - set(waits))
    bad = {k: v for k, v in waits.items() if min(v) < MIN_OUTSTANDING}
    assert not bad, bad


def test_round_wait_check_flags_a_drained_pipeline():
    # the shape of the round-2 regression: the loop head drained every load
    lines = ["_ZN11hdfs_crc32c19crc32c_tiles_kernelILi0EEEvv:", "\ts_waitcnt vmcnt(1)",
             "\tv_permlane16_swap_b32_e32 v14, v10", "\ts_waitcnt vmcnt(0) lgkmcnt(0)",
             "\tv_permlane16_swap_b32_e32 v6, v2", "\ts_endpgm"]
    kernels, waits = round_waits(lines)
    assert min(waits[next(iter(kernels))]) < MIN_OUTSTANDING


def test_product_epilogue_has_no_diagnostic_branches():
    # the store-policy experiments live in the diagnostic build's epilogue
    # (crc32c_diag_ep.h); the product kernel source compares no policy
    src = open(os.path.join(CSRC, "crc32c_kernels.hip")).read()
    code = "\n".join(line.split("//")[0] for line in src.splitlines())
    assert "store_policy ==" not in code and "kDiag && L." not in code


def test_no_noreturn_trap_in_kernels():
    # __builtin_trap() in a hot loop reshapes the CFG (see the module doc);
    # kernels fail loudly with an ordinary s_trap instead
    src = open(os.path.join(CSRC, "crc32c_kernels.hip")).read()
    code = "\n".join(line.split("//")[0] for line in src.splitlines())
    assert "__builtin_trap" not in code


def waterfall_loops(lines):
    """{kernel symbol: number of buffer memory ops sitting in a waterfall loop}:
    a buffer descriptor the compiler takes for divergent is rebuilt per
    distinct lane value -- the op is followed by `s_xor_b64 exec, exec, ...`
    and a branch back."""
    name, res = None, {}
    for i, line in enumerate(lines):
        m = re.match(r"^(_ZN11hdfs_crc32c\w+):", line)
        if m:
            name = m.group(1)
            continue
        if name and re.search(r"\bbuffer_(load|store)_", line):
            nxt = [x for x in lines[i + 1:i + 4] if x.strip() and not x.strip().startswith(";")][:1]
            if nxt and "s_xor_b64 exec, exec" in nxt[0]:
                res[name] = res.get(name, 0) + 1
    return res


def test_release_kernels_have_no_waterfall_buffer_ops(release_asm):
    """Every buffer load / store of the release kernels uses a uniform
    descriptor.  Round 3 found the device framing kernel's header staging
    built from a per-lane address: a waterfall loop that also waited for
    each of its four loads before the next (12.8 of the pass's 34 us,
    DESIGN.md §4.2)."""
    assert waterfall_loops(release_asm) == {}
