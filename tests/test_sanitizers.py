"""Host-code sanitizers: the native Avro / Kafka record-batch / HDF5 /
MQTT parsers fuzzed under ASan+UBSan, and the threaded Kafka broker + clients and the
MQTT broker + Kafka bridge + simulator under TSan.
Plain C++ harness (csrc/tests/host_sanitize.cpp), no Python extension, no GPU."""
import hashlib
import os
import shutil
import subprocess
import tempfile

import pytest

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd")
CSRC = os.path.join(PKG, "csrc")
SRCS = [os.path.join(CSRC, "tests", "host_sanitize.cpp")] + \
    [os.path.join(CSRC, "io", f) for f in ("avro.cpp", "kafka.cpp", "h5.cpp", "mqtt.cpp")]


def _build(flags, name):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    h = hashlib.sha1()
    for p in SRCS + [os.path.join(CSRC, "io", f) for f in ("avro.h", "kafka.h", "h5.h", "mqtt.h")]:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    out = os.path.join(tempfile.gettempdir(), f"sml_{name}_{h.hexdigest()[:12]}")
    if not os.path.exists(out):
        subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, *SRCS, "-o", out,
                        "-lpthread"], check=True, capture_output=True, timeout=600)
    return out


def test_codecs_fuzz_asan_ubsan():
    exe = _build(["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "asan")
    r = subprocess.run([exe, "fuzz"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "PASS fuzz" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_broker_client_threads_tsan():
    exe = _build(["-fsanitize=thread"], "tsan")
    r = subprocess.run([exe, "threads"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "PASS threads" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr


def test_checked_kernel_build_compiles_device_asserts(tmp_path):
    """SML_KERNEL_CHECKS=1 compiles SML_DCHECK into the device code; release compiles it away."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    pkg = PKG
    src = os.path.join(pkg, "csrc", "kernels", "preprocess.hip")
    outs = {}
    for flag in ("0", "1"):
        out = str(tmp_path / f"pre{flag}.s")
        subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-DSML_KERNEL_CHECKS={flag}",
                        "-I", os.path.join(pkg, "csrc", "include"), "--offload-device-only", "-S", src, "-o", out],
                       check=True, capture_output=True, timeout=300)
        outs[flag] = open(out).read()
    assert "SML_DCHECK failed" in outs["1"] and "s_trap" in outs["1"]
    assert "SML_DCHECK failed" not in outs["0"]
