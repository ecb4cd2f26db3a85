#!/usr/bin/env bash
# Build a deployable mp4x distribution (reference: bin/package.sh, which builds the shaded jar
# and zips bin/ config/ lib/ log/ into target/ytk-mp4j.zip).
#
#   bin/package.sh            -> dist/mp4x-<version>-*.whl and dist/mp4x.zip
#
# dist/mp4x.zip holds bin/ (launch scripts), config/ (logging configs), lib/ (the wheel, with
# the gfx950 native libraries inside) and an empty log/.  Offline: no build isolation, no index.
set -euo pipefail
cd "$(dirname "$0")/.."
python tools/build_native.py
rm -rf dist/mp4x
mkdir -p dist/mp4x/lib dist/mp4x/log
python -m pip wheel --no-deps --no-build-isolation --no-index -w dist/mp4x/lib . >/dev/null
cp -r bin config dist/mp4x/
( cd dist && rm -f mp4x.zip && python -m zipfile -c mp4x.zip mp4x )
ls dist/mp4x/lib
echo "dist/mp4x.zip"
