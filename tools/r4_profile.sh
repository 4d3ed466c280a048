#!/bin/bash
# Round 4's committed profiles: tools/profile_round.sh (headline and full kernel stats, FETCH/WRITE/SQ PMC passes),
# then tools/profile_hash.sh for the SHA-1 single-filter kernel and its compute-only build (shader clock under load).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/profile_round.sh &&
TAG=clock_r4 FAMS=sha1 bash tools/profile_hash.sh
