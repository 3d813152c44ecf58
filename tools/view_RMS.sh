#!/usr/bin/env bash
# Residual history of RMS-<Project>.plt with gnuplot (log scale, one curve per equation).
# Counterpart of the reference's view_RMS.sh.
#   tools/view_RMS.sh <RMS-file> [out.png]
set -euo pipefail
rms=${1:?usage: view_RMS.sh <RMS-file> [out.png]}
png=${2:-}
names=$(head -1 "$rms" | sed 's/^#VARIABLES *= *//')
IFS=',' read -r -a cols <<< "$names"
gp="$rms.gp"
{
  [ -n "$png" ] && printf 'set terminal pngcairo size 1200,700\nset output "%s"\n' "$png"
  printf 'set logscale y\nset xlabel "step"\nset ylabel "RMS"\nset grid\nplot '
  sep=""
  for ((c = 2; c <= ${#cols[@]}; c++)); do
    n=$(echo "${cols[c-1]}" | tr -d ' ')
    case "$n" in Cd*|Cv*) continue ;; esac
    printf '%s"%s" using 1:($%d > 0 ? $%d : NaN) with lines title "%s"' "$sep" "$rms" "$c" "$c" "$n"
    sep=", "
  done
  printf '\n'
  [ -z "$png" ] && printf 'pause mouse close\n'
} > "$gp"
if command -v gnuplot >/dev/null; then gnuplot "$gp"; else echo "wrote $gp (gnuplot not found)"; fi
