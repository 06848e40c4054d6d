set -o pipefail
RVC_CONV_DEBUG=0 bash scripts/pmc_conv.sh d0 "--only 4 --reps 3" || exit $?
RVC_CONV_DEBUG=7 bash scripts/pmc_conv.sh d7 "--only 4 --reps 3" || exit $?
RVC_CONV_DEBUG=0 bash scripts/pmc_conv.sh b0 "--only 4 --reps 3 --precision bf16" || exit $?
