#!/bin/bash
# Build a variant of libmppi_hip.so from the working tree with one sed expression applied to one source file
# (diagnostic A/B only): bash tools/build_variant.sh <name> <csrc file> <sed expr>  -> lib/libmppi_hip_<name>.so
set -eu
name=$1; file=$2; expr=$3
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
cp -r "$root/humanoid_mppi-rl_amd" "$root/include" "$tmp/"
rm -rf "$tmp/humanoid_mppi-rl_amd/lib"
sed -i "$expr" "$tmp/humanoid_mppi-rl_amd/csrc/$file"
if cmp -s "$tmp/humanoid_mppi-rl_amd/csrc/$file" "$root/humanoid_mppi-rl_amd/csrc/$file"; then echo "sed changed nothing"; exit 1; fi
python3 "$tmp/humanoid_mppi-rl_amd/build.py" > /dev/null
cp "$tmp/humanoid_mppi-rl_amd/lib/libmppi_hip.so" "$root/humanoid_mppi-rl_amd/lib/libmppi_hip_$name.so"
rm -rf "$tmp"
echo "built lib/libmppi_hip_$name.so"
