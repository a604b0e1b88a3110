"""CPU: resource limits of the shipped gfx950 code objects (no GPU needed).

No kernel may use scratch (private segment) memory.  A kernel with scratch,
dispatched on a queue for the first time while a persistent kernel ran on
another queue, stalled that kernel's waves for ~2 s on MI355X: the first
overlapped encoder launch of bench.py hit its dependency-wait timeout
(tools/debug_timeouts.py).  The persistent kernels' row waits are
bounded, so such a stall invalidates their output; the fix is to keep every
kernel scratch-free, and this test holds that line."""
import os
import re
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
LIBS = [os.path.join(ROOT, "webp_amd", "libwebpgpu.so")]


def code_objects(path):
    """The AMDGPU ELF code objects inside the library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        blob = open(fat, "rb").read()
    out = []
    for m in re.finditer(rb"\x7fELF\x02\x01", blob):
        o = m.start()
        if struct.unpack_from("<H", blob, o + 18)[0] != 0xE0:  # EM_AMDGPU
            continue
        shoff, = struct.unpack_from("<Q", blob, o + 0x28)
        shentsize, shnum = struct.unpack_from("<HH", blob, o + 0x3A)
        out.append(blob[o:o + shoff + shentsize * shnum])
    return out


def kernels(obj):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(obj)
        f.flush()
        txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], check=True, capture_output=True,
                             text=True).stdout
    res = {}
    for block in txt.split("  - .agpr_count")[1:]:
        name = re.search(r"\n\s+\.name:\s+(\S+)", block)
        priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
        dyn = re.search(r"\.uses_dynamic_stack:\s+(\w+)", block)
        if name and priv:
            res[name.group(1)] = (int(priv.group(1)), dyn.group(1) if dyn else "false")
    return res


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/llvm-readelf"), reason="ROCm llvm tools absent")
@pytest.mark.parametrize("lib", LIBS)
def test_no_kernel_uses_scratch(lib):
    objs = code_objects(lib)
    assert objs, "no gfx950 code object found"
    found = {}
    for o in objs:
        found.update(kernels(o))
    assert len(found) >= 20, sorted(found)
    bad = {k: v for k, v in found.items() if v[0] != 0 or v[1] != "false"}
    assert not bad, f"kernels with scratch / dynamic stack: {bad}"
