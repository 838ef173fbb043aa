#!/bin/bash
# Build a variant of libmppi_hip.so from the working tree with one sed expression applied to one source file
# (diagnostic A/B only): bash tools/build_variant.sh <name> <csrc file> <sed expr>  -> lib/libmppi_hip_<name>.so
# An empty sed expression builds the tree as it is.  VARIANT_FLAGS="<file>:<flag>[,<flag>...] ..." sets per-source hipcc flags;
# VARIANT_REV=<git rev> takes <csrc file> from that revision before the sed.
set -eu
name=$1; file=$2; expr=$3
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
cp -r "$root/humanoid_mppi-rl_amd" "$root/include" "$tmp/"
rm -rf "$tmp/humanoid_mppi-rl_amd/lib"
if [ -n "${VARIANT_REV:-}" ]; then git -C "$root" show "$VARIANT_REV:humanoid_mppi-rl_amd/csrc/$file" > "$tmp/humanoid_mppi-rl_amd/csrc/$file"; fi
if [ -n "$expr" ]; then
  sed -i "$expr" "$tmp/humanoid_mppi-rl_amd/csrc/$file"
  if cmp -s "$tmp/humanoid_mppi-rl_amd/csrc/$file" "$root/humanoid_mppi-rl_amd/csrc/$file"; then echo "sed changed nothing"; exit 1; fi
fi
if [ -n "${VARIANT_FLAGS:-}" ]; then  # merged into build.py's PER_FILE_FLAGS (replacing a file's entry)
  d=$(python3 -c 'import sys, json; print(json.dumps({f: v.split(",") for f, v in (a.split(":", 1) for a in sys.argv[1:])}))' $VARIANT_FLAGS)
  sed -i "s|^def _hipcc() -> str:|PER_FILE_FLAGS.update($d)\n\n\ndef _hipcc() -> str:|" "$tmp/humanoid_mppi-rl_amd/build.py"
  grep -q "^PER_FILE_FLAGS.update" "$tmp/humanoid_mppi-rl_amd/build.py" || { echo "flag patch failed"; exit 1; }
fi
python3 "$tmp/humanoid_mppi-rl_amd/build.py" > /dev/null
cp "$tmp/humanoid_mppi-rl_amd/lib/libmppi_hip.so" "$root/humanoid_mppi-rl_amd/lib/libmppi_hip_$name.so"
rm -rf "$tmp"
echo "built lib/libmppi_hip_$name.so"
