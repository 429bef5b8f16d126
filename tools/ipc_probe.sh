#!/bin/bash
# Runs tools/ipc_probe in pairs for every (memory kind, mode); one JSON line per rank.
cd "$(dirname "$0")"
for kind in 0 2; do
  for mode in 0 1 2; do
    d=$(mktemp -d)
    timeout -k 5 60 ./ipc_probe pair 0 "$d" $kind $mode & a=$!
    timeout -k 5 60 ./ipc_probe pair 1 "$d" $kind $mode & b=$!
    wait $a; ra=$?; wait $b; rb=$?
    echo "kind=$kind mode=$mode rc=$ra,$rb"
    rm -rf "$d"
  done
done
