#!/bin/sh
# Build the CPU oracle (test infrastructure). Outputs stay under oracle/_build/ (git-ignored).
# tests/test_oracle_sanitized.py builds the checked flavour again with ASan + UBSan
# (sanitize_main.c) and runs it over every test stream.
set -e
cd "$(dirname "$0")"
mkdir -p _build
CC=${CC:-gcc}
$CC -O2 -g -std=c11 -Wall -Wextra -fPIC -shared zflac_oracle.c -o _build/libzflac_oracle.so
$CC -O3 -march=x86-64-v4 -std=c11 -Wall -Wextra -fPIC -shared -DZFO_RELEASE_FAST zflac_oracle.c -o _build/libzflac_oracle_fast.so
