#!/bin/bash
# Build the library of another git revision (A/B baseline) into OUT.so, CPU side:
#   bash tools/build_rev.sh REV OUT.so [-DFLAG ...]
set -e
REV=$1; OUT=$(readlink -f "$2"); shift 2
TMP=$(mktemp -d /tmp/asg_rev_XXXX)
git archive "$REV" marl_sap_amd include | tar -x -C "$TMP"
(cd "$TMP" && python -m marl_sap_amd.build --out "$OUT" "$@" > /dev/null)
rm -rf "$TMP"
echo "$OUT"
