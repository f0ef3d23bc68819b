set -o pipefail
cd $GRAFT_REPO_ROOT
KT_ONLY=1 bash tools/profile.sh s58base > /dev/null 2>&1 || { echo PROF1_FAILED; exit 1; }
DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/qc1.so KT_ONLY=1 bash tools/profile.sh s58qc1 > /dev/null 2>&1 || { echo PROF2_FAILED; exit 1; }
for t in s58base s58qc1; do echo "== $t"; grep -E "k_qcells|k_cand_test|k_setup|k_join" gpurun_out/prof/$t/kt_kernel_stats.csv | cut -c1-40,100-200 | awk -F, '{print $1, $(NF-5), $(NF-4)}'; done
