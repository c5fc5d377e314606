# Build the codec library of a git revision into abx/lib_<name>.so (A/B
# against the working tree), e.g.: tools/build_ab_rev.sh r02 HEAD~3 [-DKNOB=1 ...]
set -e
name=$1; rev=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" redset_amd/csrc include | tar -x -C "$tmp"
make -s -j8 -C "$tmp/redset_amd/csrc" ../lib/libredset_hip.so \
  CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -I../../include $*"
mkdir -p "$root/abx"
cp "$tmp/redset_amd/lib/libredset_hip.so" "$root/abx/lib_$name.so"
rm -rf "$tmp"
echo "built abx/lib_$name.so from $rev"
