"""Host-code sanitizers: the native host helpers (CRC32C, TFRecord scanning, CIFAR
record gathering) driven through every entry point -- truncated and corrupt records, odd
lengths, concurrent first use -- under ASan + UBSan and under TSan. (GPU AddressSanitizer and
XNACK are not available on the MI355X pool; kernels are covered by DRN_CHECK_NAN /
DRN_DETERMINISTIC and the fp32-reference numerics tests.)"""
import shutil
import subprocess

import pytest

from distributed_resnet_tensorflow_amd.ops.build import build_host_sanitizer_driver


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("kind", ["address", "thread"])
def test_host_helpers_under_sanitizer(kind, tmp_path):
    exe = build_host_sanitizer_driver(kind, str(tmp_path))
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "host sanitizer driver: OK" in out
    assert "Sanitizer" not in out and "runtime error" not in out, out[-4000:]
