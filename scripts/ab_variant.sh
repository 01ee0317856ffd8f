#!/bin/bash
# Build a kernel variant of the extension into ab_variants/<name>/ (a copy of the package + bench.py with that .so) for
# same-box A/B runs against the in-tree build: scripts/ab_variant.sh <name> "-DDEFINE ..."
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; DEFS=$2
cd "$R"
LIPA_HIP_DEFINES="$DEFS" python -c "from llm_in_practise_amd.csrc.build import build_hip_extension as b; b()"
rm -rf "ab_variants/$NAME"; mkdir -p "ab_variants/$NAME"
cp -r llm_in_practise_amd bench.py scripts "ab_variants/$NAME/"
rm -rf "ab_variants/$NAME"/llm_in_practise_amd/__pycache__ "ab_variants/$NAME"/llm_in_practise_amd/*/__pycache__
python -c "from llm_in_practise_amd.csrc.build import build_hip_extension as b; b()"    # the in-tree build again
echo "ab_variants/$NAME ready"
