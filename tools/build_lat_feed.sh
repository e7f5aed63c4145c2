#!/bin/sh
# builds tools/bin/lat_feed against the in-tree libfws_gpu.so
cd "$(dirname "$0")/.." && mkdir -p tools/bin && \
g++ -O2 -std=c++17 -Iinclude -o tools/bin/lat_feed tools/lat_feed.cpp -Lflashws_amd/lib -lfws_gpu \
    -Wl,-rpath,'$ORIGIN/../../flashws_amd/lib'
