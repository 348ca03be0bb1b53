"""Compile every HIP source for gfx950 to assembly and list our kernels that spill VGPRs or use scratch
(``.private_segment_fixed_size`` > 0): spills in a hot kernel are a silent 2-5x.  Usage: python tools/spill_audit.py"""
import concurrent.futures as cf
import re
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import build_ext as b  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]


def _bad(name: str, info: dict) -> bool:
    """VGPR spills or scratch in our own kernels (SGPR spills land in VGPR lanes: cheap; rocPRIM's are not ours)."""
    if "rocprim" in name:
        return False
    return bool(info.get("vgpr_spill_count", 0) or info.get("private_segment_fixed_size", 0))


def audit(src: Path, out_dir: Path) -> list:
    inc, _, abi = b._torch_paths()
    s = out_dir / (src.stem + ".s")
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-munsafe-fp-atomics", "-mllvm", "-amdgpu-kernarg-preload-count=16",
           *[f"-I{p}" for p in inc], f"-I{ROOT / 'csrc'}", "--cuda-device-only", "-S", "-o", str(s), str(src)]
    if src.suffix == ".cpp":
        cmd[1:1] = ["-x", "hip"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return [(src.name, "COMPILE FAILED", r.stderr[-300:])]
    rows, name, info = [], None, {}
    for line in s.read_text().splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            if name and _bad(name, info):
                rows.append((src.name, name, dict(info)))
            name, info = m.group(1), {}
            continue
        m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count|vgpr_count):\s+(\d+)", line)
        if m and name:
            info[m.group(1)] = int(m.group(2))
    if name and _bad(name, info):
        rows.append((src.name, name, dict(info)))
    return rows


def main():
    srcs = sorted((ROOT / "csrc").rglob("*.hip"))
    with tempfile.TemporaryDirectory() as d, cf.ThreadPoolExecutor(4) as ex:
        results = list(ex.map(lambda p: audit(p, Path(d)), srcs))
    n = 0
    for rows in results:
        for f, k, info in rows:
            n += 1
            print(f"{f}: {k[:110]} {info}")
    print(f"{n} kernels with spills / scratch in {len(srcs)} sources")


if __name__ == "__main__":
    main()
