# Build a variant of the engine with the product flags plus extra ones:
#   bash tools/build_variant.sh OUT.so [extra hipcc flags...]
set -e
cd "$(dirname "$0")/.."
OUT=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-sched-strategy=max-ilp \
  -Iinclude "$@" -o "$OUT" phylostan_amd/csrc/phylo_hip.hip
