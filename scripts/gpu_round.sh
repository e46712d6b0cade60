# One GPU call: tests + smoke + benches (scripts/gpu_tests.sh), then the rocprof pass (profile.sh).
set -o pipefail
bash scripts/gpu_tests.sh || exit $?
bash scripts/profile.sh ${1:-r02}
