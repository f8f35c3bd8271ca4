#!/bin/bash
# Build an A/B variant of libmarlnav.so into marl-nav_amd/lib/<name>.so, from
# the working tree with extra -D flags, or from a git revision:
#   scripts/build_variant.sh ref HEAD             # the committed kernels
#   scripts/build_variant.sh ntoff "" -DMARLNAV_NT_STORES=0
# then: LIBS=marl-nav_amd/lib/ref.so bash scripts/cmd_ab.sh (on the GPU box)
set -eu
cd "$(dirname "$0")/../marl-nav_amd/csrc"
name=$1 rev=${2:-}
shift $(( $# >= 2 ? 2 : 1 ))
src=marlnav_step.hip
if [ -n "$rev" ]; then
    git show "$rev:marl-nav_amd/csrc/marlnav_step.hip" > .variant_step.hip
    src=.variant_step.hip
fi
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -ffp-contract=off \
    -Wno-pass-failed "$@" "$src" marlnav_rollout.hip -o "../lib/$name.so"
rm -f .variant_step.hip
echo "built marl-nav_amd/lib/$name.so"
