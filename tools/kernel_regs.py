"""Per-kernel register / LDS / spill figures of a built object (dgvcc_amd/build/<file>.o), from the
gfx950 code object's AMDGPU metadata notes.

usage: python tools/kernel_regs.py conv [name-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernels(obj: str):
    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "k.co")
        fb = os.path.join(d, "fb.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
                               check=True).stdout
        dem = subprocess.run(["c++filt"], input=notes, capture_output=True, text=True).stdout
    out = []
    for blk in re.split(r"\n\s+- \.agpr_count:", dem)[1:]:
        def g(k):
            m = re.search(rf"\.{k}:\s+(\S+)", blk)
            return m.group(1) if m else "?"
        name = re.search(r"\.name:\s+(.+)", blk).group(1).strip()
        agpr = blk.split("\n", 1)[0].strip()
        out.append((name, g("vgpr_count"), agpr, g("sgpr_count"), g("group_segment_fixed_size"),
                    g("vgpr_spill_count"), g("sgpr_spill_count")))
    return out


if __name__ == "__main__":
    f = sys.argv[1] if len(sys.argv) > 1 else "conv"
    obj = os.path.join(ROOT, "dgvcc_amd", "build", f + ".o")
    pats = sys.argv[2:]
    print(f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'lds':>7} {'vspill':>6} {'sspill':>6}  kernel")
    for k in kernels(obj):
        if pats and not any(p in k[0] for p in pats):
            continue
        print(f"{k[1]:>5} {k[2]:>5} {k[3]:>5} {k[4]:>7} {k[5]:>6} {k[6]:>6}  {k[0]}")
