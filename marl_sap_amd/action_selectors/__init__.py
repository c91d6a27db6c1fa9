"""Action selector registry (reference: action_selectors/__init__.py)."""
from .classic_selectors import EpsilonGreedyActionSelector, MultinomialActionSelector, SoftPoliciesSelector
from .sap_selectors import EpsilonGreedySAPTestActionSelector, SequentialAssignmentProblemSelector
from .lsa import linear_sum_assignment_batched

REGISTRY = {
    "multinomial": MultinomialActionSelector,
    "epsilon_greedy": EpsilonGreedyActionSelector,
    "soft_policies": SoftPoliciesSelector,
    "sap": SequentialAssignmentProblemSelector,
    "epsilon_greedy_sap_test": EpsilonGreedySAPTestActionSelector,
}
