"""Reference constants for the ``one_model_att`` path (oracle side; test infrastructure).

Every value cites the reference line it is read from; paths are relative to
``/root/reference/MADDPG_ownENV_randomOD_radar_one_model_att/`` (``ATT/`` in SURVEY.md).
"""

DT = 0.5                 # env_simulator.time_step                      ATT/env:57, :201
ACC_MAX = 8              # acc_max                                       ATT/main:136
VMAX = 5                 # max_spd -> Agent.maxSpeed                      ATT/main:150, ATT/agent:34
PB = 2.5                 # Agent.protectiveBound (radius)                 ATT/agent:43
DETECTION_RANGE = 30     # Agent.detectionRange (diameter)                ATT/agent:41
RADAR_DIST = DETECTION_RANGE / 2   # radar_dist = detectionRange / 2       ATT/env:1066
N_RAYS = 18              # range(0, 360, 20)                              ATT/env:1062
BOUND = (455, 680, 255, 385)  # xlow, xhigh, ylow, yhigh                  ATT/params:32-36
GRID_LEN = 10            # gridLength                                     ATT/grid:138
EPISODE_LENGTH = 50      # --episode_length                               ATT/main:918
GOAL_RADIUS = 1          # Point(goal[-1]).buffer(1)                      ATT/env:2266
WP_REACH = 5             # wp_reach_threshold_dist                        ATT/env:2276
CRASH_PENALTY = 20       # crash_penalty_wall                             ATT/env:2115
REACH_REWARD = 20        # reach_target                                   ATT/env:2121
NEAR_LO = 2.5            # dist_to_penalty_lowerbound                     ATT/env:2422
NEAR_HI = 10             # dist_to_penalty_upperbound                     ATT/env:2420
GAMMA = 0.95             # GAMMA                                          ATT/params:27
TAU = 0.01               # TAU                                            ATT/params:28
LR = 0.001               # actorNet_lr / criticNet_lr                     ATT/main:139-140
EPS_END = 8000           # eps_end (noise schedule)                       ATT/main:169
MEMORY_LENGTH = int(1e5)  # --memory_length                               ATT/main:920
GRU_HISTORY = 10         # gru_history_length (push starts once full)     ATT/main:130, :363

# quadSegs = 16 is shapely's buffer default; GEOS filletAngleQuantum = pi/2/quadSegs.
QUAD_SEGS = 16
MATH_PI = 3.14159265358979323846  # GEOS MATH_PI (== math.pi)

# normalisation constants, NormalizeData(bound[0:2], bound[2:4], max_spd, acc_range)  ATT/env:87
X_SCALE = (1 - (-1)) / (BOUND[1] - BOUND[0])   # ATT/util:567
Y_SCALE = (1 - (-1)) / (BOUND[3] - BOUND[2])   # ATT/util:568


def d0_of(n_agents):
    """Own-observation width 6 + 4(N-1)  (canonical contract R1)."""
    return 6 + 4 * (n_agents - 1)
