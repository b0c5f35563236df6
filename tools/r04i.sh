#!/bin/bash
# Round-4 check: GPU suite + bench + kernel trace (tools/r04_check.sh), then
# the pass-2 tile-start profile and the wave-rotation A/B.
bash tools/r04_check.sh r04g || exit $?
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/sp2_prof.sh r04g_sp2 sp2prof || exit $?
bash tools/sp2_prof.sh r04g_sp2 rotprof || exit $?
bash tools/variant_ab.sh r04g_ab 2 default rot || exit $?
