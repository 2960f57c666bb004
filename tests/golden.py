"""Golden cases, derived from the reference semantics main.cu:40-89,377-397."""
PATH5 = (5, [(0, 1), (1, 2), (2, 3), (3, 4)])
CASES = [
    # (graph, groups, expected F, expected report k (1-based), expected min F)
    (PATH5, [[0], [2], [0, 4]], [10, 6, 4], 3, 4),
    (PATH5, [[4], [1, 3], [3, 1], [0]], [10, 3, 3, 10], 2, 3),           # tie -> lowest index
    (PATH5, [[2], [], [99, -1]], [6, 0, 0], 2, 0),                        # empty / out of range
    ((6, [(0, 1), (1, 2), (3, 4)]), [[0], [3], [5]], [3, 1, 0], 3, 0),    # unreachable not counted
    ((3, [(0, 0), (0, 1), (0, 1), (1, 2)]), [[0]], [3], 1, 3),            # self-loop, duplicates
    (PATH5, [], [], 0, -1),                                               # K = 0
]
