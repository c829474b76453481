"""The reference's experiment-JSON surface, read for the engine.

Field names and defaults mirror
  Config            /root/reference/src/algorithm/tools/utils.py:14-20
  PolicyOptions     /root/reference/src/algorithm/policies.py:31-34
  ModelOptions      /root/reference/src/algorithm/policies.py:36-41
  optimizer_options /root/reference/src/algorithm/nic_nes/experiment.py:20-21
A leading underscore disables a key ("_from_infos"), as in the reference JSON files. The engine
implements the mscoco_nes.json hot path only: net 'fc_caption', every Fitness value (greedy, the
greedy_* criteria, and the sampled sample / self_critical / sc_loss), model_options.safe_mutations
'' / SM-G-SUM / SM-VECTOR / SM-PROPORTIONAL (nicnes.mutations), no vbn / layer_n; anything else
raises NotSupported (nicnes_create returns NICNES_ERR_UNSUPPORTED for unsupported model sizes).
"""
import json
from collections import namedtuple

config_fields = [
    'l2coeff', 'noise_stdev', 'stdev_divisor', 'eval_prob', 'snapshot_freq', 'log_dir',
    'batch_size', 'patience', 'val_batch_size', 'num_val_batches',
    'num_val_items', 'cuda', 'max_nb_iterations', 'ref_batch_size', 'bs_multiplier', 'stepsize_divisor',
    'single_batch', 'schedule_limit', 'schedule_start'
]
Config = namedtuple('Config', field_names=config_fields, defaults=(None,) * len(config_fields))

_opt_fields = ['net', 'safe_mutations', 'model_options', 'safe_mutation_underflow', 'fitness',
               'vbn', 'safe_mutation_batch_size', 'safe_mutation_vector']
PolicyOptions = namedtuple('PolicyOptions', field_names=_opt_fields,
                           defaults=[None, '', {}, 0.01, None, False, 32, None])

_model_opt_fields = ['vocab_size', 'input_encoding_size', 'rnn_type', 'rnn_size', 'num_layers',
                     'drop_prob_lm', 'seq_length', 'fc_feat_size', 'vbn', 'vbn_e', 'vbn_affine', 'layer_n',
                     'layer_n_affine', 'safe_mutation_underflow', 'safe_mutations', 'safe_mutation_vector',
                     'safe_mutation_batch_size']
ModelOptions = namedtuple('ModelOptions', field_names=_model_opt_fields, defaults=(0,) * len(_model_opt_fields))


# Fitness modes the engine implements: greedy decoding, scored by CIDEr-D alone or by a criterion
# over the greedy tokens' log-probs (Fitness.is_greedy, src/captioning/policies.py:45-47)
GREEDY_FITNESS = ('greedy', 'greedy_logprob', 'greedy_expprob', 'greedy_linprob', 'greedy_avgprob')
SAMPLED_FITNESS = ('sample', 'self_critical', 'sc_loss')
FITNESS = GREEDY_FITNESS + SAMPLED_FITNESS          # every Fitness enum value (src/captioning/policies.py:22-35)


class NotSupported(ValueError):
    pass


def load_experiment(path_or_dict):
    """JSON file or dict -> dict with disabled ('_'-prefixed) top-level keys dropped."""
    exp = path_or_dict
    if not isinstance(exp, dict):
        with open(path_or_dict) as f:
            exp = json.load(f)
    return {k: v for k, v in exp.items() if not k.startswith('_')}


class ExperimentSpec:
    """What the engine needs from an experiment JSON (mscoco_nes.json and variants)."""

    def __init__(self, exp, vocab_size=9487, seq_length=16):
        exp = load_experiment(exp)
        if exp.get('algorithm', 'nic_nes') != 'nic_nes':
            raise NotSupported('algorithm %r: the engine implements nic_nes' % exp.get('algorithm'))
        if exp.get('dataset', 'mscoco') != 'mscoco':
            raise NotSupported('dataset %r: the engine implements the mscoco fc_caption path' % exp.get('dataset'))
        self.exp = exp
        self.config = Config(**exp['config'])
        po = dict(exp['policy_options'])
        self.policy_options = PolicyOptions(**po)
        mo = dict(po.get('model_options', {}))
        mo.setdefault('vocab_size', vocab_size)          # injected from data, captioning/experiment.py:27-30
        mo.setdefault('seq_length', seq_length)
        self.model_options = ModelOptions(**{k: v for k, v in mo.items() if k in _model_opt_fields})
        self._validate()
        opt = exp.get('optimizer_options', {'type': 'adam', 'args': {'stepsize': 1e-3}})
        self.optimizer_type = opt['type']
        self.optimizer_args = dict(opt.get('args', {}))
        if self.optimizer_type not in ('adam', 'sgd'):
            raise NotSupported('optimizer %r' % self.optimizer_type)
        self.nb_offspring = int(exp.get('nb_offspring', 1))

    def _validate(self):
        po, mo = self.policy_options, self.model_options
        if po.net != 'fc_caption':
            raise NotSupported('net %r: the engine implements fc_caption' % po.net)
        if self.fitness not in FITNESS:
            raise NotSupported("fitness %r: the engine implements %s (src/captioning/policies.py:22-61)"
                               % (po.fitness, ', '.join(FITNESS)))
        if po.vbn or mo.vbn_e or mo.layer_n:
            raise NotSupported('virtual batch norm / layer norm are not implemented by the engine')
        m = self.mutation
        if m == 'SM-G-ABS':
            raise NotSupported("SM-G-ABS: the reference's _calc_abs_sensitivity raises AttributeError "
                               "(self.nb_params on Sensitivity, safe_mutations.py:125)")
        if m not in ('', 'SM-G-SUM', 'SM-VECTOR', 'SM-PROPORTIONAL'):
            raise NotSupported('safe_mutations %r (Mutation, src/algorithm/nets.py:16-21)' % m)

    # ------------------------------------------------------------------------------------
    @property
    def fitness(self):
        """policy_options.fitness; Fitness.DEFAULT is 'greedy' (policies.py:35)."""
        return self.policy_options.fitness or 'greedy'

    @property
    def mutation(self):
        """model_options.safe_mutations: the option the network reads (Mutation(options.safe_mutations),
        nets.py:46); policy_options.safe_mutations is not read by the reference's nets."""
        return self.model_options.safe_mutations or ''

    @property
    def single_batch(self):
        """config.single_batch: True = every member on the task's one batch; falsy (the reference's
        default, and mscoco_nes.json's false) = every member on its own batch, as each reference
        worker draws one per member (nic_nes_worker.py:121-128)."""
        return bool(self.config.single_batch)

    @property
    def batches_per_iteration(self):
        """Distinct batches per iteration: 1 with single_batch, else one per member, capped by the
        engine-only key 'batches_per_iteration' (members then share batches round-robin)."""
        if self.single_batch:
            return 1
        cap = int(self.exp.get('batches_per_iteration') or self.nb_offspring)
        return max(1, min(self.nb_offspring, cap))

    @property
    def sigma(self):
        return float(self.config.noise_stdev)

    @property
    def batch_size(self):
        return int(self.config.batch_size)

    @property
    def l2coeff(self):
        return float(self.config.l2coeff or 0.0)

    def engine_kwargs(self, max_members, noise_len=1 << 27, noise_seed=0, max_batch=None):
        mo = self.model_options
        return dict(vocab_size=int(mo.vocab_size), input_encoding_size=int(mo.input_encoding_size or 128),
                    rnn_size=int(mo.rnn_size or 128), fc_feat_size=int(mo.fc_feat_size or 2048),
                    seq_length=int(mo.seq_length or 16), max_batch=int(max_batch or self.batch_size),
                    max_members=int(max_members), noise_len=int(noise_len), noise_seed=int(noise_seed))
