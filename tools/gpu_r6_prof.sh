# r6 rocprof evidence: kernel trace + stats, FETCH_SIZE / WRITE_SIZE / SQ passes of the bench
set -o pipefail
bash profiles/run_profiles.sh r6
