# round-4 GPU pass 2: drop-in tests and the default bench
set -o pipefail
ROUND=r04 bash tools/gpu_round.sh dropin bench
