#!/usr/bin/env bash
# Colour map of one variable of a Tecplot POINT field file (<Project>.plt, tp-<Project>.plt)
# with gnuplot.  Counterpart of the reference's viewplt.sh.
#   tools/viewplt.sh <file.plt> [variable=Mach] [zone=last] [out.png]
# Without gnuplot on PATH it only writes <file>.<var>.gp and <file>.<var>.dat.
set -euo pipefail
plt=${1:?usage: viewplt.sh <file.plt> [variable] [zone] [out.png]}
var=${2:-Mach}
zone=${3:-last}
png=${4:-}
col=$(awk -v v="$var" 'toupper($0) ~ /^ *VARIABLES/ {
        sub(/^[^=]*=/, ""); n = split($0, a, ",");
        for (i = 1; i <= n; i++) { gsub(/[ "]/, "", a[i]); if (a[i] == v) { print i; exit } } }' "$plt")
[ -n "$col" ] || { echo "variable '$var' not in $plt" >&2; exit 1; }
nz=$(grep -ci '^ *ZONE' "$plt")
[ "$zone" = last ] && zone=$nz
stem="$plt.$var"
# zone <zone> only, one blank line whenever Y changes (gnuplot grid rows)
awk -v z="$zone" 'toupper($0) ~ /^ *ZONE/ { k++; next } toupper($0) ~ /^ *(VARIABLES|TITLE)/ { next }
     k == z && NF { if (seen && $2 != y) print ""; y = $2; seen = 1; print }' "$plt" > "$stem.dat"
{
  [ -n "$png" ] && printf 'set terminal pngcairo size 1600,600\nset output "%s"\n' "$png"
  printf 'set view map\nset pm3d map\nset size ratio -1\nset xlabel "X, mm"\nset ylabel "Y, mm"\n'
  printf 'set title "%s (zone %s of %s)"\nsplot "%s" using 1:2:%s with pm3d notitle\n' "$var" "$zone" "$nz" "$stem.dat" "$col"
  [ -z "$png" ] && printf 'pause mouse close\n'
} > "$stem.gp"
if command -v gnuplot >/dev/null; then gnuplot "$stem.gp"; else echo "wrote $stem.gp (gnuplot not found)"; fi
