"""The tile kernel's image-reference scan (policy-server_amd/csrc/imgscan.hpp, compiled for the host
from the same source the kernel includes) equals a byte loop restating the normalisation rules:
tests/imgscan_check.cpp."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = next((c for c in ("/opt/rocm/llvm/bin/clang++", shutil.which("clang++") or "") if c and os.path.exists(c)), None)


@pytest.mark.skipif(CLANG is None, reason="no clang++ (ext_vector_type)")
def test_image_scan_matches_byte_loop(tmp_path):
    exe = tmp_path / "imgscan_check"
    subprocess.run([CLANG, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "policy-server_amd", "csrc"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "imgscan_check.cpp")], check=True)
    out = subprocess.run([str(exe), "300000"], check=False, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout
