"""The host sanitizer run (tests/sanitize/run.sh): libbsdc_io (BAM codec + C++ family formation)
and oracle/ rebuilt with ASan + UBSan, and the corrupt / truncated / malformed BAM tests and the
family-formation parity tests run against them.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan")
def test_codec_and_oracle_clean_under_asan_ubsan():
    p = subprocess.run([os.path.join(ROOT, "tests", "sanitize", "run.sh"), "-k",
                        "corrupt or truncated or malformed or round_trip or family_image or golden or numpy or "
                        "forced_large or split_partner or empty_input or restatement or stand_in"],
                       capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "sanitizer builds loaded" in p.stdout and " passed" in p.stdout
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr
