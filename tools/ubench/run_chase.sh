#!/bin/bash
# loaded-latency sweep of tools/ubench/chase (each run bounded)
cd "$(dirname "$0")"
for mib in 16 64 256 1024 4096; do
  for w in 1 6; do
    timeout -k 5 60 ./chase $mib $w 1 200 || exit 1
  done
  timeout -k 5 60 ./chase $mib 6 2 200 || exit 1
done
timeout -k 5 60 ./chase 1024 6 1 200 2048 || exit 1
timeout -k 5 60 ./chase 1024 6 1 200 65536 || exit 1
timeout -k 5 60 ./chase 4096 8 1 200 || exit 1
