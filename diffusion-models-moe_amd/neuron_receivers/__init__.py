"""Drop-in receiver API of the reference's `neuron_receivers` package (hot-path receivers only).

Importing this package requires the sdmoe HIP library at call time (no CPU path). Skill-discovery receivers of
the reference (frequency/expert statistics, Wanda column norms, bounding boxes, HPO variants) are outside this
tier and are not exported.
"""
from neuron_receivers.base_receiver import BaseNeuronReceiver, GEGLU, GELU  # noqa: F401
from neuron_receivers.predictivity import NeuronPredictivity  # noqa: F401
from neuron_receivers.moefy import MOEFy  # noqa: F401
from neuron_receivers.remove_skilled_experts import RemoveExperts  # noqa: F401
from neuron_receivers.remove_wanda_neurons_fast import WandaRemoveNeuronsFast  # noqa: F401
from neuron_receivers.multi_concept_remover import MultiConceptRemoverWanda  # noqa: F401
