#!/bin/bash
# Build the HIP library from the working tree into tools/exp/<name>.so (an A/B
# variant for tools/ab_variants.sh); the in-tree product library is untouched.
# VARIANT_FLAGS adds compiler flags (e.g. -DABNN_ABLATE_FILTER=1 for an
# experiment compiled only into the variant).
set -e
name=${1:?usage: tools/build_variant.sh NAME}
cd "$(dirname "$0")/.."
mkdir -p tools/exp
python3 - "$name" <<'PY'
import os, sys
from abnn_amd import build as b
out = os.path.join("tools", "exp", sys.argv[1] + ".so")
extra = os.environ.get("VARIANT_FLAGS", "").split()
b.build_hip(out=out, defines=extra)
print(out)
PY
