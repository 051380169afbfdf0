"""No hot HIP kernel may spill to scratch.

A scratch access is a round trip to memory (hundreds of cycles); one struct that the
compiler failed to promote to registers cost the reference-LSTM trainer a global load per
Adam block this round.  This test reads every gfx950 code object bundled in the built
`_C.so` (the `.hip_fatbin` section: one offload bundle per translation unit) and checks
each kernel's `.private_segment_fixed_size` in the AMDGPU metadata notes.  CPU only: it
needs the built extension and the ROCm LLVM tools, not a GPU.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd")
LLVM = "/opt/rocm/lib/llvm/bin/"
SO = os.path.join(PKG, "_C.so")

# Kernels allowed a private segment: the fully dynamic dense-AE fallback (runtime
# activation codes, unvectorised loads) -- never taken by the reference models, which
# compile their activations in (PACK_REF).
ALLOWED = (r"ae_train_kernelILin1ELb0ELi0ELi3E",)


def _kernel_scratch(so_path, tmp_path):
    fb = tmp_path / "fatbin.bin"
    subprocess.run([LLVM + "llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", so_path, str(tmp_path / "x.so")],
                   check=True, capture_output=True)
    data = fb.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)]
    sizes = {}
    for i, st in enumerate(starts):
        end = starts[i + 1] if i + 1 < len(starts) else len(data)
        b, o = tmp_path / f"b{i}.bin", tmp_path / f"b{i}.o"
        b.write_bytes(data[st:end])
        subprocess.run([LLVM + "clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={b}", f"--output={o}"],
                       check=True, capture_output=True)
        notes = subprocess.run([LLVM + "llvm-readelf", "--notes", str(o)], check=True, capture_output=True,
                               text=True).stdout
        name = None
        for line in notes.splitlines():
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
                continue
            m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
            if m and name:
                sizes[name] = int(m.group(1))
                name = None
    return sizes


@pytest.mark.skipif(not os.path.exists(SO) or not shutil.which(LLVM + "llvm-readelf"),
                    reason="built _C.so and ROCm LLVM tools needed")
def test_no_hot_kernel_uses_scratch(tmp_path):
    sizes = _kernel_scratch(SO, tmp_path)
    assert len(sizes) > 100, f"found only {len(sizes)} kernels in the bundled code objects"
    for must in ("lstm_ref_train_b1_kernel", "lstm_serve_ref1_kernel", "ae_minibatch", "ae_serve"):
        assert any(must in k for k in sizes), f"{must} not among the bundled kernels"
    bad = {k: v for k, v in sizes.items() if v and not any(re.search(p, k) for p in ALLOWED)}
    assert not bad, f"kernels with a private (scratch) segment: {bad}"
