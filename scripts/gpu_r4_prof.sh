set -o pipefail
cd /root/repo
export TMPDIR=/tmp
ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/prof.so timeout -k 10 300 python3 scripts/phase_profile.py --B 65536 > gpurun_out/r4_prof_new.txt 2>&1 || { tail -20 gpurun_out/r4_prof_new.txt; exit 1; }
cat gpurun_out/r4_prof_new.txt
ACL_PROF_OLDPACK=1 ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/prof3.so timeout -k 10 300 python3 scripts/phase_profile.py --B 65536 > gpurun_out/r4_prof_old.txt 2>&1 || { tail -20 gpurun_out/r4_prof_old.txt; exit 1; }
cat gpurun_out/r4_prof_old.txt
