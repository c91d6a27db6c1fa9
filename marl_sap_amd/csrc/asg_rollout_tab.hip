// asg_rollout_tab.hip -- the rollout kernel instances of the float64-table benefit modes
// (MT19937 compat, injected sat_prox_mat): asg_h2.hip compiled for launch_rollout_tab only.
#define ASG_H2_TU 1
#include "asg_h2.hip"
