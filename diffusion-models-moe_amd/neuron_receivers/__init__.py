"""Drop-in receiver API of the reference's `neuron_receivers` package.

Importing this package requires the sdmoe HIP library at call time (no CPU path). Hot-path receivers (MOEFy,
RemoveExperts, WandaRemoveNeuronsFast, MultiConceptRemoverWanda) plus the two discovery receivers that produce
their inputs (GetExperts -> expert lists, Wanda -> column norms -> masks). The remaining
statistics/HPO receivers of the reference are not exported.
"""
from neuron_receivers.base_receiver import BaseNeuronReceiver, GEGLU, GELU  # noqa: F401
from neuron_receivers.predictivity import NeuronPredictivity  # noqa: F401
from neuron_receivers.moefy import MOEFy  # noqa: F401
from neuron_receivers.remove_skilled_experts import RemoveExperts  # noqa: F401
from neuron_receivers.remove_wanda_neurons_fast import WandaRemoveNeuronsFast  # noqa: F401
from neuron_receivers.multi_concept_remover import MultiConceptRemoverWanda  # noqa: F401
from neuron_receivers.get_experts import GetExperts  # noqa: F401
from neuron_receivers.wanda_receiver import Wanda  # noqa: F401
