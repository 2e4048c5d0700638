set -o pipefail
bash tools/pmc.sh s6c2 --scene c2 --reps 2 '{"bvh":2}'; echo rc=$?
