"""Action selector registry (reference: action_selectors/__init__.py)."""
from .bet_selectors import ContinuousActionSelector
from .classic_selectors import EpsilonGreedyActionSelector, MultinomialActionSelector, SoftPoliciesSelector
from .filtered_selectors import (FilteredEpsGrSAPTestActionSelector, FilteredEpsilonGreedyActionSelector,
                                 FilteredSAPActionSelector, FilteredSoftPoliciesSelector)
from .sap_selectors import EpsilonGreedySAPTestActionSelector, SequentialAssignmentProblemSelector
from .lsa import linear_sum_assignment_batched

REGISTRY = {
    "continuous": ContinuousActionSelector,
    "multinomial": MultinomialActionSelector,
    "epsilon_greedy": EpsilonGreedyActionSelector,
    "soft_policies": SoftPoliciesSelector,
    "sap": SequentialAssignmentProblemSelector,
    "epsilon_greedy_sap_test": EpsilonGreedySAPTestActionSelector,
    "filtered_const_sap": FilteredSAPActionSelector,
    "filtered_const_epsilon_greedy": FilteredEpsilonGreedyActionSelector,
    "filtered_const_epsgr_sap_test": FilteredEpsGrSAPTestActionSelector,
    "filtered_const_soft_policies": FilteredSoftPoliciesSelector,
}
