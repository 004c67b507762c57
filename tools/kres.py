"""Per-kernel resources of the built library (VGPRs, spills, scratch, LDS) from its gfx950 code object:
    python tools/kres.py [LIB.so] [NAME-FILTER]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = "/opt/rocm/lib/llvm/bin"
lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "sdfgenfast_amd", "libsdfgen_hip.so")
flt = sys.argv[2] if len(sys.argv) > 2 else "sweep_tile"
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={d}/fat.bin", lib], check=True)
    subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={d}/fat.bin",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={d}/k.co"], check=True)
    notes = subprocess.run([f"{B}/llvm-readelf", "--notes", f"{d}/k.co"], capture_output=True, text=True).stdout
# one kernel's metadata: a '- .args:' list item up to the next one
recs = re.split(r"\n  - \.agpr_count:", notes)
for r in recs:
    f = dict(re.findall(r"\n\s+\.(name|vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|"
                        r"group_segment_fixed_size):\s+(\S+)", r))
    if flt in f.get("name", ""):
        nm = subprocess.run(["c++filt"], input=f["name"], capture_output=True, text=True).stdout.strip()
        nm = nm.replace("sdfhip::", "").replace("k_sweep_tile", "tile")
        print(f"{nm[:90]:90s} vgpr {f.get('vgpr_count')} vspill {f.get('vgpr_spill_count')} sspill "
              f"{f.get('sgpr_spill_count')} scratch {f.get('private_segment_fixed_size')} lds {f.get('group_segment_fixed_size')}")
