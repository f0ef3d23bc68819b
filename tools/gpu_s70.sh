set -o pipefail
cd $GRAFT_REPO_ROOT
KT_ONLY=1 bash tools/profile.sh s70nt > /dev/null 2>&1 || { echo PROF1_FAILED; exit 1; }
DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/nt0.so KT_ONLY=1 bash tools/profile.sh s70base > /dev/null 2>&1 || { echo PROF2_FAILED; exit 1; }
echo done
