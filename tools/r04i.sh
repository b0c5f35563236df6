#!/bin/bash
# Round-4 check: GPU suite + bench + kernel trace (tools/r04_check.sh) on the
# product library (sparse pass-2 schedule), then the pass-2 tile-start
# profile and an A/B of the schedule against the round-3 one (old) and its
# group sizes (rows16 / rows4) and the wave rotation (rot).
bash tools/r04_check.sh r04g || exit $?
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/sp2_prof.sh r04g_sp2 sp2prof || exit $?
bash tools/variant_ab.sh r04g_ab 2 default old rows16 rows4 rot || exit $?
