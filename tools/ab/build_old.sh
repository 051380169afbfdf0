#!/usr/bin/env bash
# Build the committed (HEAD) kernels into tools/ab/_C_old.so for ab_ae.sh / ab.sh, then
# rebuild the working tree's _C.so.  CPU only (hipcc cross-compiles).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
P=hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd
T=$(mktemp -d)
git diff --name-only HEAD -- "$P/csrc" > "$T/changed"
while read -r f; do mkdir -p "$T/$(dirname "$f")"; cp "$f" "$T/$f"; done < "$T/changed"
git checkout HEAD -- $(cat "$T/changed")
python -c "from streamml import _build; _build.build_all(verbose=False, checked=False)"
cp "$P/_C.so" tools/ab/_C_old.so
while read -r f; do cp "$T/$f" "$f"; done < "$T/changed"
python -c "from streamml import _build; _build.build_all(verbose=False, checked=False)"
rm -rf "$T"
echo "old = $(git rev-parse --short HEAD); changed: $(tr '\n' ' ' < /dev/null)"
