"""Register budgets of the C4 item kernels, read from the built gfx950 code object (no GPU).

The v-mode items run two 1024-lane workgroups per CU, i.e. 8 waves per SIMD; the SGPR file admits
that only while a wave's SGPR granule, ceil(sgpr_count / 16) * 16 + 16, is at most 96 (800 SGPRs
per SIMD; /opt/skills/guides/MI355X_MICROARCH.md, "Residency").  One added kernel argument once
took .sgpr_count past 80 and the v-mode launch from 69 to 113 ms (one item per CU); the 512-lane
u-mode items (four per CU) fall from 4 to 3 per CU at the same edge.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "cypher-for-apache-spark_amd", "build", "k_tri.o")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(obj, tmp):
    """{kernel name: (sgpr_count, vgpr_count, group_segment_fixed_size)} from the object's notes."""
    fat, co = os.path.join(tmp, "k.fatbin"), os.path.join(tmp, "k.co")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, obj, os.path.join(tmp, "o")],
                   check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fat,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True, capture_output=True)
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    out = {}
    for block in re.split(r"\n  - \.agpr_count:", notes)[1:]:
        name = re.search(r"\n    \.name:\s+(\S+)", block).group(1)
        sg = int(re.search(r"\n    \.sgpr_count:\s+(\d+)", block).group(1))
        vg = int(re.search(r"\n    \.vgpr_count:\s+(\d+)", block).group(1))
        out[name] = (sg, vg)
    return out


@pytest.mark.skipif(not os.path.exists(OBJ) or not os.path.exists(os.path.join(LLVM, "llvm-readelf")),
                    reason="k_tri.o not built or no ROCm llvm tools")
def test_item_kernels_keep_two_items_per_cu(tmp_path):
    ks = _kernels(OBJ, str(tmp_path))
    items = {k: v for k, v in ks.items() if "k_tri_big_items" in k or "k_tri_items_sp" in k}
    assert items, "no k_tri_big_items kernels in the object"
    assert any("k_tri_items_sp" in k for k in items), "no split-list item kernels in the object"
    for name, (sg, vg) in items.items():
        # k_tri_big_items<U, VM, B> / k_tri_items_sp<U, VM, B, ...>: the list walks (every instantiation is a
        # product path since round 6 removed the flat walk and the 8 / 16-load A/B variants)
        m = re.search(r"k_tri_(?:big_items|items_sp)ILi(\d+)ELb(\d)ELi(\d+)E", name)
        assert m, name
        granule = -(-sg // 16) * 16 + 16
        waves = 800 // granule
        need = 8  # 2 x 1024 lanes or 4 x 512 lanes per CU = 8 waves per SIMD
        assert waves >= need, f"{name}: sgpr_count {sg} admits {waves} waves per SIMD, need {need}"
        assert vg * need <= 512, f"{name}: {vg} VGPRs"
