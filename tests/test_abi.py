"""CPU tests of the C-ABI boundary: the library builds, loads, exports every
symbol include/*.h declares, and fails loudly (no CPU fallback) without a GPU."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", src)
    return sorted(set(n for n in names if n not in ("sizeof",)))


@pytest.fixture(scope="module")
def libpath():
    from hadoofus_amd import build
    return build.build()


def test_headers_compile_as_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "crc32c.h"\n#include "hadoofus_crc32c.h"\n'
                   "int main(void){ return (int)sizeof(hdfs_crc32c_segment) - 48; }\n")
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           "-c", str(src), "-o", str(tmp_path / "t.o")])


@pytest.fixture(scope="module")
def diagpath(libpath):
    from hadoofus_amd import build
    return build.DIAG_LIB


def _exported(path):
    """Defined dynamic symbols, version suffixes (name@@NODE) stripped."""
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    return set(l.split()[-1].split("@")[0] for l in out.splitlines() if l.strip())


def test_release_has_no_diagnostic_knobs(libpath, diagpath):
    """The release library exports none of include/hadoofus_crc32c_diag.h and
    reads none of the tuning variables (the strings are not even in it); the
    diagnostic build exports and reads them all."""
    diag_decl = set(_declared("hadoofus_crc32c_diag.h"))
    assert {"hdfs_crc32c_set_store_policy", "hdfs_crc32c_probe_read", "hdfs_crc32c_set_tile_order"} <= diag_decl
    assert not diag_decl & _exported(libpath)
    assert diag_decl <= _exported(diagpath)
    rel = open(libpath, "rb").read()
    dia = open(diagpath, "rb").read()
    for var in (b"HDFS_CRC32C_STORE", b"HDFS_CRC32C_TILE_ORDER", b"HDFS_CRC32C_NT", b"HDFS_CRC32C_DEPTH",
                b"HDFS_CRC32C_STREAMS", b"HDFS_CRC32C_BLOCK", b"HDFS_CRC32C_GROUP", b"HDFS_CRC32C_ALIGN",
                b"HDFS_CRC32C_SMALL_RULE", b"HDFS_CRC32C_XCD", b"HDFS_CRC32C_RUNS"):
        assert var not in rel, var
        assert var in dia, var


def test_release_kernels_are_the_product_shapes(libpath, diagpath):
    """The release build's tiled kernels are the two product shapes (schedule
    3 with buffer loads, schedule 2) in their product variants only: compute
    and verify, each with and without the realigning path for byte-unaligned
    data, verify also with the fused copy-out -- twelve in all -- plus
    compute on schedule 3 with the LDS group gather; no load-only twin
    (mode 2), no schedule 4 and no read probes.  The diagnostic build has
    them."""
    import re as _re
    rel = open(libpath, "rb").read()
    dia = open(diagpath, "rb").read()
    pat = (rb"_ZN11hdfs_crc32c19crc32c_tiles_kernelILi(\d)ELi(\d)ELi(\d)ELi(\d)ELi(\d)ELi(\d+)ELi(\d)ELi(\d)"
           rb"ELi(\d)ELi(\d)EEE")
    shapes = set(_re.findall(pat, rel))
    variants = [(b"0", b"0", b"0"), (b"0", b"0", b"1")] + [(b"1", cp, un) for cp in (b"0", b"1") for un in (b"0", b"1")]
    want = {(m, o, b"1", b"3", b"1", b"1024", buf, cp, un, b"0") for m, cp, un in variants
            for o, buf in ((b"3", b"1"), (b"2", b"0"))}
    want.add((b"0", b"3", b"1", b"3", b"1", b"1024", b"1", b"0", b"0", b"1"))  # compute: LDS group gather
    assert shapes == want, shapes ^ want
    assert b"probe_read_kernel" not in rel and b"probe2_kernel" not in rel
    dshapes = set(_re.findall(pat, dia))
    assert any(s[0] == b"2" for s in dshapes) and len(dshapes) > 20
    assert b"probe_read_kernel" in dia


def test_exports_every_declared_symbol(libpath):
    exported = _exported(libpath)
    for h in ("crc32c.h", "hadoofus_crc32c.h"):
        decl = _declared(h)
        assert decl, h
        missing = [d for d in decl if d not in exported]
        assert not missing, (h, missing)
    # the reference drop-in trio (src/crc32c.h:13,17,24)
    for n in ("_hdfs_crc32c", "_hdfs_sse42_crc32c", "_hdfs_sw_crc32c"):
        assert n in exported


def test_exports_nothing_else(libpath):
    """Built with -fvisibility=hidden: the only exported functions are the
    declared C ABI (HIP kernel host stubs are exported by the toolchain)."""
    out = subprocess.check_output(["nm", "-D", "--defined-only", libpath], text=True)
    decl = set(_declared("crc32c.h")) | set(_declared("hadoofus_crc32c.h"))
    extra = []
    for line in out.splitlines():
        parts = line.split()
        if len(parts) < 3 or parts[1] not in "TW":
            continue
        name = parts[2].split("@")[0]
        if name in decl or name in ("_init", "_fini", "HADOOFUS_CRC32C_%d" % _abi_version()):
            continue
        if name.startswith("_ZN11hdfs_crc32c") and "_kernel" in name:
            continue
        extra.append(name)
    assert not extra, extra


def test_packet_struct_layout():
    import ctypes

    from hadoofus_amd.abi import Packet
    assert ctypes.sizeof(Packet) == 56


def test_segment_struct_layout():
    import ctypes

    from hadoofus_amd.abi import Segment
    assert ctypes.sizeof(Segment) == 48
    assert Segment.crcs.offset == 32 and Segment.bitmap.offset == 40


def test_no_cpu_fallback_without_gpu(libpath):
    """Without a usable gfx950 the engine reports ENODEV, and the total
    drop-in function aborts loudly instead of computing on the CPU."""
    code = (
        "import ctypes,sys\n"
        f"lib=ctypes.CDLL({libpath!r})\n"
        "lib.hdfs_crc32c_init.restype=ctypes.c_int\n"
        "rc=lib.hdfs_crc32c_init(-1)\n"
        "if rc==0: sys.exit(3)\n"  # a GPU is present: not this test's scenario
        "assert rc==-2, rc\n"
        "lib._hdfs_crc32c.restype=ctypes.c_uint32\n"
        "lib._hdfs_crc32c.argtypes=[ctypes.c_uint32,ctypes.c_char_p,ctypes.c_uint]\n"
        "lib._hdfs_crc32c(0,b'123456789',9)\n"
        "sys.exit(0)\n")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="-1")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    if p.returncode == 3:
        pytest.skip("a GPU is visible")
    assert p.returncode != 0, "drop-in returned a value with no GPU (silent fallback?)"
    assert "engine unavailable" in p.stderr


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "hadoofus_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dp, f)).read()
                assert "oracle" not in txt.replace("no oracle", ""), f


def build_consumer(tmp_path, libpath):
    """Compile + link the drop-in consumer (tests/consumer/t_unit_dropin.c)."""
    exe = tmp_path / "t_unit_dropin"
    libdir = os.path.dirname(libpath)
    subprocess.check_call(["gcc", "-std=gnu99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "consumer", "t_unit_dropin.c"), "-o", str(exe),
                           "-L", libdir, "-Wl,-rpath," + libdir, "-lhadoofus_crc32c"])
    import json
    kats = json.load(open(os.path.join(ROOT, "tests", "golden", "kats.json")))["kats"]
    txt = tmp_path / "kats.txt"
    txt.write_text("".join(f"{k['len']} {k['crc']:08x} {k['hex'] or '-'}\n" for k in kats))
    return exe, txt


def build_c(tmp_path, libpath, name):
    """Compile + link tests/consumer/<name>.c against the engine."""
    exe = tmp_path / name
    libdir = os.path.dirname(libpath)
    subprocess.check_call(["gcc", "-std=gnu99", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "consumer", name + ".c"), "-o", str(exe),
                           "-L", libdir, "-Wl,-rpath," + libdir, "-lhadoofus_crc32c"])
    return exe


def test_packet_consumer_links(tmp_path, libpath):
    assert build_c(tmp_path, libpath, "packet_consumer").exists()


def test_dropin_consumer_links(tmp_path, libpath):
    exe, txt = build_consumer(tmp_path, libpath)
    assert exe.exists() and txt.read_text().count("\n") >= 7


def test_struct_layouts_match_c(tmp_path):
    """ctypes mirrors of the public structs have the C layout (gcc, the
    reference's compiler)."""
    import ctypes

    from hadoofus_amd.abi import OutPacket, Packet, Segment
    src = tmp_path / "l.c"
    src.write_text(
        '#include <stddef.h>\n#include <stdio.h>\n#include "hadoofus_crc32c.h"\n'
        "int main(void){ printf(\"%zu %zu %zu %zu %zu %zu\\n\", sizeof(hdfs_crc32c_out_packet),"
        " offsetof(hdfs_crc32c_out_packet, data_len), offsetof(hdfs_crc32c_out_packet, crc_len),"
        " offsetof(hdfs_crc32c_out_packet, last), sizeof(hdfs_crc32c_packet), sizeof(hdfs_crc32c_segment));"
        " return 0; }\n")
    exe = tmp_path / "l"
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                           "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)], text=True).split()]
    assert got == [ctypes.sizeof(OutPacket), OutPacket.data_len.offset, OutPacket.crc_len.offset,
                   OutPacket.last.offset, ctypes.sizeof(Packet), ctypes.sizeof(Segment)]


def test_both_libraries_load_and_bind(libpath, diagpath):
    """Both builds dlopen with every symbol resolved (RTLD_NOW, as the
    diagnostic build is loaded by tools and tests on the GPU box) and bind
    every function their headers declare."""
    from hadoofus_amd import abi
    mode = os.RTLD_NOW | os.RTLD_LOCAL
    abi.bind_product(ctypes.CDLL(libpath, mode=mode))
    abi.bind_diag(abi.bind_product(ctypes.CDLL(diagpath, mode=mode)))


def _signature_sections():
    """tests/golden/abi_signatures.txt -> {version: {name: prototype}}."""
    sec, cur = {}, None
    with open(os.path.join(ROOT, "tests", "golden", "abi_signatures.txt")) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line or line.startswith("#"):
                continue
            if line.startswith("["):
                cur = int(line.strip("[]"))
                sec[cur] = {}
                continue
            name, proto = line.split(": ", 1)
            sec[cur][name] = proto
    return sec


def _abi_version():
    txt = open(os.path.join(ROOT, "include", "hadoofus_crc32c.h")).read()
    return int(re.search(r"#define HDFS_CRC32C_ABI_VERSION (\d+)", txt).group(1))


def test_header_prototypes_are_the_committed_abi():
    """The headers' prototypes are exactly the committed list of the current
    ABI version, and no function of it kept a name an earlier version gave a
    different signature: a caller built against another version fails to
    bind instead of passing shifted arguments (round 3 broke this rule:
    verify_packets_copy gained two arguments in the middle under the same
    name, and a tool holding the round-2 prototype crashed -- DESIGN 10.1)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import abi_signatures
    sec = _signature_sections()
    v = _abi_version()
    assert max(sec) == v, (sorted(sec), v)
    assert abi_signatures.header_prototypes() == sec[v]
    for old in sec:
        if old == v:
            continue
        for name, proto in sec[v].items():
            if name in sec[old]:
                assert sec[old][name] == proto, (name, old, sec[old][name], proto)


def test_exports_carry_the_version_node(libpath, diagpath):
    """Every exported engine symbol (the C ABI and the drop-in trio) is in the
    version node HADOOFUS_CRC32C_<ABI version> of exports.map."""
    v = _abi_version()
    for path in (libpath, diagpath):
        out = subprocess.check_output(["objdump", "-T", path], text=True)
        seen = {}
        for line in out.splitlines():
            parts = line.split()
            if len(parts) >= 3 and (parts[-1].startswith("hdfs_crc32c_") or parts[-1].startswith("_hdfs_")):
                seen[parts[-1]] = parts[-2]
        assert "hdfs_crc32c_read_packets" in seen and "_hdfs_crc32c" in seen
        bad = {n: ver for n, ver in seen.items() if ver != f"HADOOFUS_CRC32C_{v}"}
        assert not bad, bad
    assert "hdfs_crc32c_verify_packets_copy" not in _exported(libpath)


def test_abi_version_call_and_binding_check(libpath):
    """hdfs_crc32c_abi_version() needs no GPU and equals the header's
    version; the Python bindings refuse a library of another version."""
    from hadoofus_amd import abi
    lib = ctypes.CDLL(libpath)
    lib.hdfs_crc32c_abi_version.restype = ctypes.c_int
    assert lib.hdfs_crc32c_abi_version() == _abi_version() == abi.ABI_VERSION

    class Old:
        @staticmethod
        def hdfs_crc32c_abi_version():
            return 3
    with pytest.raises(ImportError):
        abi.check_abi(Old())
