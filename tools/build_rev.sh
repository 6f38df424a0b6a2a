# build the library of git revision REV into geomesa_amd/lib/NAME.so (same-box A/B against the working tree)
#   bash tools/build_rev.sh REV NAME [-DDEFINE ...]
set -e
rev=$1; name=$2; shift 2
tmp=$(mktemp -d)
git -C "$(dirname "$0")/.." archive "$rev" geomesa_amd include | tar -x -C "$tmp"
out=$(cd "$(dirname "$0")/.." && pwd)/geomesa_amd/lib/$name.so
(cd "$tmp" && python -m geomesa_amd.build --force --out="$out" "$@" > /dev/null)
rm -rf "$tmp"
echo "$out"
