# Build an experiment variant of libmpcmmd.so from a patched copy of the
# sources (the product sources stay untouched):
#   bash tools/variant.sh TAG 'python-expression editing s (the text of k_betacem.hip etc.)' [file]
# -> mpc-mmd_amd/libmpcmmd_TAG.so  (compare with MPCMMD_LIB=... on the GPU box)
set -e
TAG=$1
EXPR=$2
FILE=${3:-k_betacem.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/mpcmmd_variant_$TAG
rm -rf $W && mkdir -p $W && cp -r $ROOT/mpc-mmd_amd $ROOT/include $W/
python3 - "$W/mpc-mmd_amd/csrc/$FILE" "$EXPR" <<'PY'
import sys
p, e = sys.argv[1], sys.argv[2]
s = open(p).read()
t = eval(e, {"s": s})
assert t != s, "variant expression changed nothing"
open(p, "w").write(t)
PY
rm -rf $W/mpc-mmd_amd/build $W/mpc-mmd_amd/*.so
make -s -C $W/mpc-mmd_amd -j8 >/dev/null
cp $W/mpc-mmd_amd/libmpcmmd.so $ROOT/mpc-mmd_amd/libmpcmmd_$TAG.so
echo built mpc-mmd_amd/libmpcmmd_$TAG.so
