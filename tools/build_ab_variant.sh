# Build a variant of the codec library into abx/lib_<name>.so with extra
# compile definitions, e.g.: tools/build_ab_variant.sh memonly -DREDSET_MEMONLY=1
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
cp -r "$root/redset_amd" "$root/include" "$tmp/"
rm -rf "$tmp/redset_amd/build" "$tmp/redset_amd/lib" "$tmp/redset_amd/bin"
make -s -j8 -C "$tmp/redset_amd/csrc" ../lib/libredset_hip.so \
  CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -I../../include $*"
mkdir -p "$root/abx"
cp "$tmp/redset_amd/lib/libredset_hip.so" "$root/abx/lib_$name.so"
rm -rf "$tmp"
echo "built abx/lib_$name.so"
