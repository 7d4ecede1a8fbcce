"""Properties of the built gfx950 code objects (CPU only: the library is disassembled, nothing runs)."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "pyorbslam_amd" / "_lib" / "liborbfe.so"
OBJDUMP = Path("/opt/rocm/lib/llvm/bin/llvm-objdump")


def _disassembly(tmp_path):
    if not LIB.exists() or not OBJDUMP.exists():
        pytest.skip("liborbfe.so or llvm-objdump missing")
    lib = tmp_path / "liborbfe.so"
    shutil.copy(LIB, lib)  # --offloading writes the bundles next to its input
    subprocess.run([str(OBJDUMP), "--offloading", str(lib)], cwd=tmp_path, check=True, capture_output=True)
    objs = sorted(tmp_path.glob("liborbfe.so.*gfx950*"))
    assert objs, "no gfx950 code object in liborbfe.so"
    return "\n".join(subprocess.run([str(OBJDUMP), "-d", str(o)], check=True, capture_output=True,
                                    text=True).stdout for o in objs)


def _functions(dis):
    """{symbol: body} of every kernel in the disassembly."""
    out, name, body = {}, None, []
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            if name:
                out[name] = "\n".join(body)
            name, body = m.group(1), []
        elif name:
            body.append(line)
    if name:
        out[name] = "\n".join(body)
    return out


def test_m0_only_for_writelane(tmp_path):
    """k_orb keeps its four ballots with v_writelane_b32 whose lane select the inline asm puts in M0, a
    register the compiler does not preserve across asm: no other instruction of such a kernel may read
    or write M0."""
    funcs = _functions(_disassembly(tmp_path))
    users = {n: b for n, b in funcs.items() if "v_writelane_b32" in b}
    assert any("k_orb" in n for n in users), "k_orb no longer uses v_writelane_b32: update this test"
    for n, b in users.items():
        for line in b.splitlines():
            if re.search(r"\bm0\b", line):
                ins = line.split("//")[0].split()
                op = next((t for t in ins if re.match(r"^[sv]_|^ds_|^buffer_|^global_", t)), "")
                assert op in ("s_mov_b32", "v_writelane_b32"), f"{n}: unexpected M0 use: {line.strip()}"


def test_product_library_reads_no_environment():
    """no environment variable can change a kernel path of the production library —
    it imports no getenv and names no ORBFE_* variable (the development knobs of earlier rounds live only in
    tools/dbg/build_variant.sh builds, ORBFE_DEV_VARIANTS)."""
    if not LIB.exists():
        pytest.skip("liborbfe.so missing")
    und = subprocess.run(["nm", "-D", "--undefined-only", str(LIB)], check=True, capture_output=True, text=True).stdout
    assert not re.search(r"\b(secure_)?getenv\b", und), "liborbfe.so imports getenv"
    strs = subprocess.run(["strings", str(LIB)], check=True, capture_output=True, text=True).stdout
    names = set(re.findall(r"\bORBFE_[A-Z0-9_]+\b", strs)) - {"ORBFE_NSTAGES"}
    assert not names, f"liborbfe.so names environment-style knobs: {sorted(names)}"


def test_gpu_push_carries_no_dev_variant_libraries():
    """the tree gpurun pushes (tar with .gpurunignore's patterns) holds no development
    variant library (pyorbslam_amd/_lib/variants/, tools/dbg/build_variant.sh builds) and still holds the
    product library and the oracle checker the GPU runs load."""
    if not shutil.which("tar"):
        pytest.skip("tar missing")
    r = subprocess.run(["tar", "-cvf", "/dev/null", "--exclude=./.git", "--exclude-from=.gpurunignore", "."],
                       cwd=ROOT, check=True, capture_output=True, text=True)
    names = [n.strip() for n in r.stdout.splitlines()]
    assert not [n for n in names if "/_lib/variants" in n], "dev variant libraries travel to the GPU box"
    if LIB.exists():
        assert "./pyorbslam_amd/_lib/liborbfe.so" in names
    assert "./bench.py" in names and "./tests/golden/" in names


def test_buffer_resources_built_only_by_the_helpers():
    """Every buffer resource of the kernels is built by uniform_rsrc / bounded_rsrc / aligned_rsrc, which pass the
    address halves through uint32_t: __builtin_amdgcn_readfirstlane returns int, and an ad-hoc construction that
    OR-ed its sign-extended low half into the 64-bit base corrupted the high address bits whenever bit 31 of
    the address was set (round 6: two GPU faults on the 4 500-px batch test)."""
    src = (ROOT / "pyorbslam_amd" / "csrc" / "orbfe_kernels.hip").read_text()
    helpers = {"uniform_rsrc", "bounded_rsrc", "aligned_rsrc"}
    current, offenders = None, []
    for i, line in enumerate(src.splitlines(), 1):
        m = re.match(r"^__device__ __forceinline__ __amdgpu_buffer_rsrc_t (\w+)\(", line)
        if m:
            current = m.group(1)
        elif re.match(r"^\S", line):
            current = None
        if "__builtin_amdgcn_make_buffer_rsrc" in line and current not in helpers:
            offenders.append(i)
    assert not offenders, f"buffer resources built outside the helpers at lines {offenders}"
