#!/bin/bash
# Build an A/B variant of libmarlnav.so into marl-nav_amd/lib/<name>.so, from
# the working tree with extra -D flags, or from a git revision:
#   scripts/build_variant.sh ref HEAD        # the committed kernels
#   scripts/build_variant.sh exp "" -DSOME_TIMING_SWITCH=1
# then: LIBS=marl-nav_amd/lib/ref.so bash scripts/cmd_ab.sh (on the GPU box)
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name=$1 rev=${2:-}
shift $(( $# >= 2 ? 2 : 1 ))
src="$ROOT"
tmp=""
if [ -n "$rev" ]; then
    tmp=$(mktemp -d)
    git -C "$ROOT" archive "$rev" marl-nav_amd/csrc include | tar -x -C "$tmp"
    src="$tmp"
fi
cd "$src/marl-nav_amd/csrc"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -ffp-contract=off \
    -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-kernarg-preload-count=14 -Wno-pass-failed "$@" marlnav_step.hip marlnav_rollout.hip -o "$ROOT/marl-nav_amd/lib/$name.so"
[ -n "$tmp" ] && rm -rf "$tmp"
echo "built marl-nav_amd/lib/$name.so"
