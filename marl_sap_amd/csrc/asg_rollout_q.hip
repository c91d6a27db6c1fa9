// asg_rollout_q.hip -- the rollout kernel instances that write the agent's Q rows instead of
// selecting (asg_step_forward, both benefit sources): asg_h2.hip compiled for launch_rollout_q only.
#define ASG_H2_TU 2
#include "asg_h2.hip"
