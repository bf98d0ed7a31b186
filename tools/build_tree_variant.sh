#!/usr/bin/env bash
# Build the native library of another git revision for tools/abvariant.py:
#   bash tools/build_tree_variant.sh NAME REV
# -> tools/variants/NAME/libingot_gpu.so (ingot_amd/csrc + include at REV).
# DEFS (optional) adds compiler defines, e.g. DEFS=-DINGOT_EMIT_UNROLL=8.
# REV = WORKTREE builds the working tree's sources instead.
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2
src=tools/build/tree_$name
rm -rf "$src"; mkdir -p "$src/ingot_amd/csrc" "$src/include" tools/variants/$name
if [[ $rev == WORKTREE ]]; then
    cp -r ingot_amd/csrc/. "$src/ingot_amd/csrc/"; cp -r include/. "$src/include/"
else
    git archive "$rev" ingot_amd/csrc include | tar -x -C "$src"
fi
objs=()
for f in "$src"/ingot_amd/csrc/*.hip "$src"/ingot_amd/csrc/*.cpp; do
    o="$src/$(basename "$f").o"
    x=(); [[ $f == *.cpp ]] && x=(-x hip)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function \
        "${x[@]}" ${DEFS:-} -I"$src/include" -c "$f" -o "$o" &
    objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/$name/libingot_gpu.so "${objs[@]}"
echo "built tools/variants/$name/libingot_gpu.so from $rev"
