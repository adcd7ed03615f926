# Build the engine library of a git revision (or the working tree, "wt") into ab/lib<name>.so
# for A/B timing on one GPU box (tools/ab.sh).  usage: [AB_DEFS=-DX=1] tools/ab_build.sh <name> [rev | wt | dir]
set -euo pipefail
root=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=${2:-wt}
mkdir -p "$root/ab"
if [ "$rev" = wt ]; then
  src=$root
elif [ -d "$rev" ]; then  # a directory holding clonos_amd/ and include/
  src=$rev
else
  src=/tmp/ab_wt_$name; rm -rf "$src"; mkdir -p "$src"
  git -C "$root" archive "$rev" clonos_amd include | tar -x -C "$src"
fi
objs=()
for f in engine.cpp kernels.hip decode_fast.hip decode_fused.hip replay.hip encode.hip response.cpp; do
  o=/tmp/ab_${name}_$f.o
  /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w ${AB_DEFS:-} -I "$src/include" -c "$src/clonos_amd/csrc/$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/ab/lib$name.so" "${objs[@]}"
echo "$root/ab/lib$name.so"
