. "$(dirname "$0")/common.sh"
TAG=${1:-r6i}
timeout -k 10 200 python scripts/sac_phase_timing.py --variant cur --batch 256 --steps 300 --out "$O/sac_phases_${TAG}_b256.json" \
  > "$O/sac_phases_${TAG}_b256.log" 2>&1; hard $? phases
echo DONE
