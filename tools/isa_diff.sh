#!/bin/bash
# Compare the gfx950 instruction streams of two builds of the codec objects
# (redset_amd/build/*.o): extract each object's .hip_fatbin, unbundle the
# gfx950 code object, disassemble without addresses and raw bytes, diff.
# usage: tools/isa_diff.sh <dir of old .o files> <dir of new .o files>
set -euo pipefail
B=/opt/rocm/lib/llvm/bin
old=$1 new=$2 tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
for o in "$old"/*.o; do
  f=$(basename "$o" .o)
  [ -f "$new/$f.o" ] || { echo "MISSING $f"; continue; }
  for tag in old new; do
    src=$([ $tag = old ] && echo "$old/$f.o" || echo "$new/$f.o")
    objcopy --dump-section .hip_fatbin="$tmp/$tag.fatbin" "$src" 2>/dev/null || { echo "NOFATBIN $f"; continue 2; }
    $B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$tmp/$tag.fatbin" \
      --output="$tmp/$tag.co" --unbundle
    $B/llvm-objdump -d --no-show-raw-insn "$tmp/$tag.co" | grep -v "file format" |
      sed -E 's/^\s*[0-9a-f]+:\s*//; s/\s*\/\/.*$//' > "$tmp/$tag.s"
  done
  if cmp -s "$tmp/old.s" "$tmp/new.s"; then echo "SAME $f ($(wc -l < "$tmp/old.s") lines)"
  else echo "DIFF $f ($(diff "$tmp/old.s" "$tmp/new.s" | grep -c '^[<>]') lines differ)"; fi
done
