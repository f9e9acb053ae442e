# rocprof kernel times of the stats build for env variants (timing dissection)
export PA_LIBRARY=$GRAFT_REPO_ROOT/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd/libpa_stats.so
bash $GRAFT_REPO_ROOT/scripts/prof_env.sh
