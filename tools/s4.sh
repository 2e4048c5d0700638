set -o pipefail
bash tools/pmc.sh s4c2 --scene c2 --reps 2 '{"bvh":0}'; echo rc=$?
