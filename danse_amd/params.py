"""Run/config API of the reference, kept field-for-field.

Mirrors the dataclasses a user of the reference configures:
``DANSEparameters`` (``danse_toolbox/d_base.py:145-391``),
``CohDriftParameters`` (``d_base.py:55-110``), ``PrintoutsAndPlotting``
(``d_base.py:120-143``), ``PreComputedFilters`` (``d_base.py:22-37``),
``WASNparameters`` / ``TopologyParameters`` / ``RandomIRParameters`` /
``RandomSignalsParameters`` (``siggen/classes.py:16-376``, the fields the
engine and the offline scene path use), ``ExportParameters`` /
``TestParameters`` (``danse_toolbox/d_classes.py:133-324``) and the YAML
loader ``load_from_yaml`` (``danse_toolbox/dataclass_methods.py:258-329``).

Same names, same defaults, same ``__post_init__`` validation (ValueError on
invalid config), so a reference YAML file loads unchanged.  Interactive
``input()`` prompts of the reference are replaced by the ValueError branch.
"""
from __future__ import annotations

import ast
import copy
import random
from dataclasses import dataclass, field, fields, is_dataclass

import numpy as np
import yaml


@dataclass
class PreComputedFilters:
    active: bool = False
    internalFilters: list = field(default_factory=list)
    externalFilters: list = field(default_factory=list)
    filtersCentr: list = field(default_factory=list)
    filtersLocal: list = field(default_factory=list)
    filtersSSBC: list = field(default_factory=list)
    purpose: str = 'noise-only'   # 'noise-only' | 'speech-only'


@dataclass
class CohDriftParameters:
    alpha: float = .95
    segLength: int = 10
    estEvery: int = 1
    startAfterNups: int = 11
    estimationMethod: str = 'gs'
    alphaEps: float = .05
    loop: str = 'closed'


@dataclass
class PrintoutsAndPlotting:
    verbose: bool = True
    showWASNs: bool = False
    printout_batch_updates: bool = True
    printout_profiler: bool = True
    printout_eventsParser: bool = True
    printout_eventsParserNoBC: bool = False
    printout_externalFilterUpdate: bool = True

    def __post_init__(self):
        self.printout_eventsParser = self.printout_eventsParser and self.verbose
        self.printout_eventsParserNoBC = self.printout_eventsParserNoBC and self.verbose
        self.printout_profiler = self.printout_profiler and self.verbose
        self.printout_externalFilterUpdate = self.printout_externalFilterUpdate and self.verbose


def get_divisors(n):
    n = int(n)
    return sorted({d for i in range(1, int(n ** 0.5) + 1) if n % i == 0 for d in (i, n // i)})


@dataclass
class DANSEparameters:
    # Hyperparameters (d_base.py:112-118)
    efficientSpSBC: bool = True
    bypassUpdates: bool = False
    # General
    simType: str = 'batch'
    maxBatchUpdates: int = 10
    DFTsize: int = 1024
    WOLAovlp: float = .5
    updateEvery: int = 1
    nodeUpdating: str = 'seq'
    seqUpdateStartNodeIdx: int = 0
    broadcastType: str = 'wholeChunk'
    broadcastLength: float = None
    winWOLAanalysisType: str = 'sqrthann'
    winWOLAsynthesisType: str = 'sqrthann'
    upTDfilterEvery: float = 1.
    noFusionAtSingleSensorNodes: bool = False
    # SROs
    compensateSROs: bool = False
    includeFSDflags: bool = True
    estimateSROs: str = 'Oracle'
    compensationStrategy: str = 'node-specific'
    cohDrift: CohDriftParameters = field(default_factory=CohDriftParameters)
    # Filter update
    performGEVD: bool = False
    GEVDrank: int = 1
    noExternalFilterRelaxation: bool = False
    timeBtwExternalFiltUpdates: float = 0.
    onlyBroadcastRefSensorSigs: bool = False
    alphaExternalFilters: float = 1.
    t_expAvg50pExternalFilters: float = 2.
    t_expAvg50p: float = 2.
    forcedBeta: float = None
    forcedBetaExternalFilters: float = None
    filterInitType: str = 'selectFirstSensor'
    filterInitFixedValue: float = 0.
    # SCM initialisation
    covMatInitType: str = 'fully_random'
    covMatEyeInitScaling: float = 1.
    covMatRandomInitScaling: float = float(np.finfo(float).eps)
    covMatSameInitForAllNodes: bool = True
    covMatSameInitForAllFreqs: bool = True
    use1stFrameAsBasis: bool = False
    printoutsAndPlotting: PrintoutsAndPlotting = field(default_factory=PrintoutsAndPlotting)
    # Desired signal estimation
    desSigProcessingType: str = 'wola'
    computeLocal: bool = False
    computeCentralised: bool = False
    computeSingleSensorBroadcast: bool = False
    # Metrics (kept for config compatibility; evaluation is out of scope)
    gammafwSNRseg: float = 0.2
    frameLenfwSNRseg: float = 0.03
    minNoSpeechDurEndUtterance: float = 0.2
    startComputeMetricsAt: str = 'beginning_2nd_utterance'
    endComputeMetricsAt: str = None
    preGivenFilters: PreComputedFilters = field(default_factory=PreComputedFilters)
    # TI-DANSE (out of scope; fields kept so YAML files load)
    treeFormationAlgorithm: str = 'prim'
    keepOriginalTree: bool = False
    # Debugging
    saveConditionNumber: bool = False
    saveConditionNumberEvery: int = 1
    wasnInfoInitiated: bool = False
    startUpdatesAfterAtLeast: float = 0.

    def __post_init__(self):
        """``d_base.py:332-380``."""
        self.printoutsAndPlotting.__post_init__()
        self.Ns = int(self.DFTsize * (1 - self.WOLAovlp))
        self.winWOLAanalysis = _window(self.winWOLAanalysisType, self.DFTsize, self.WOLAovlp, 'analysis')
        self.winWOLAsynthesis = _window(self.winWOLAsynthesisType, self.DFTsize, self.WOLAovlp, 'synthesis')
        self.normFactWOLA = self.Ns / sum(self.winWOLAanalysis)
        if self.broadcastType == 'wholeChunk':
            self.broadcastLength = self.Ns
        elif self.broadcastType == 'fewSamples' and self.broadcastLength is None:
            self.broadcastLength = 1
        elif self.broadcastType == 'fewSamples' and self.broadcastLength is not None:
            if self.broadcastLength > self.Ns:
                raise ValueError(f'Broadcast length ({self.broadcastLength}) cannot be larger than the WOLA frame size ({self.Ns}).')
            if self.Ns % self.broadcastLength != 0:
                raise ValueError(f'Broadcast length ({self.broadcastLength}) must be a divisor of the WOLA frame size ({self.Ns}). Possible divisors: {get_divisors(self.Ns)}.')
        if self.estimateSROs not in ['Oracle', 'CohDrift', 'DXCPPhaT']:
            raise ValueError(f'The field "estimateSROs" accepts values ["Oracle", "CohDrift", "DXCPPhaT"]. Current value: "{self.estimateSROs}".')
        if self.noExternalFilterRelaxation:
            self.timeBtwExternalFiltUpdates = 0.
        if self.simType not in ['batch', 'online']:
            raise ValueError(f'Unknown simulation type: {self.simType}. Valid values: ["batch", "online"].')
        self.compensationStrategy = self.compensationStrategy.lower()
        if self.compensationStrategy not in ['network-wide', 'node-specific']:
            raise ValueError(f'Unknown compensation strategy: {self.compensationStrategy}. Valid values: ["network-wide", "node-specific"].')

    def get_wasn_info(self, wasnParams: 'WASNparameters'):
        """``d_base.py:382-391``."""
        self.nNodes = wasnParams.nNodes
        self.nSensorPerNode = wasnParams.nSensorPerNode
        self.referenceSensor = wasnParams.referenceSensor
        self.baseFs = wasnParams.fs
        self.seed = wasnParams.topologyParams.seed
        self.wasnInfoInitiated = True


def _window(kind, n, ovlp, which):
    if kind == 'sqrthann':
        return np.sqrt(np.hanning(n))   # symmetric Hann (quirk Q8)
    if kind == 'rect':
        return np.ones(n)
    if kind == 'rect_normNs':
        return np.ones(n) * np.sqrt(ovlp)
    raise ValueError(f'Unknown {which} window type: {kind}')


@dataclass
class RandomIRParameters:
    distribution: str = 'uniform'
    minValue: float = -.5
    maxValue: float = .5
    duration: float = 0.2
    decay: str = 'none'
    decayTimeConstant: float = 0.1


@dataclass
class RandomSignalsParameters:
    distribution: str = 'uniform'
    minValue: float = -1.
    maxValue: float = 1.
    pauseType: str = 'none'
    pauseDuration: float = 0.5
    pauseSpacing: float = 0.5
    randPauseDuration_max: float = 0.5
    randPauseDuration_min: float = 0.1
    randPauseSpacing_max: float = 0.5
    randPauseSpacing_min: float = 0.1
    startWithPause: bool = False


@dataclass
class TopologyParameters:
    topologyType: str = 'fully-connected'
    commDistance: float = 0.
    seed: int = 12345
    plotTopo: bool = False
    userDefinedTopo: np.ndarray = field(default_factory=lambda: np.array([]))

    def __post_init__(self):
        pass


@dataclass
class WASNparameters:
    """Fields of ``siggen.classes.WASNparameters`` (``siggen/classes.py:66-376``)."""
    trueRoom: bool = True
    randIRsParams: RandomIRParameters = field(default_factory=RandomIRParameters)
    rd: np.ndarray = field(default_factory=lambda: np.array([5, 5, 5]))
    fs: float = 16000.
    t60: float = 0.
    minDistToWalls: float = 0.5
    layoutType: str = 'random'
    predefinedLayoutFile: str = ''
    spinTop_randomWiggleAmount: float = 0.0
    spinTop_minInterNodeDist: float = None
    spinTop_minSourceSpacing: float = None
    referenceSensor: int = 0
    interSensorDist: float = 0.1
    arrayGeometry: str = 'grid3d'
    lenRIR: int = 2 ** 10
    sigDur: float = 5.
    diffuseNoise: bool = False
    diffuseNoisePowerFactor: float = 0.
    typeDiffuseNoise: str = 'noise'
    fileDiffuseBabble: str = ''
    nDesiredSources: int = 1
    nNoiseSources: int = 1
    signalType: str = 'from_file'
    desiredSignalFile: list = field(default_factory=list)
    noiseSignalFile: list = field(default_factory=list)
    randSignalsParams: RandomSignalsParameters = field(default_factory=RandomSignalsParameters)
    noiseSignalFilesLoadedFromFolder: str = None
    snrBasis: str = 'dry_signals'
    snr: int = 5
    VADenergyDecrease_dB: float = 30
    VADwinLength: float = 20e-3
    vadMinProportionActive: float = 0.5
    enableVADloadFromFile: bool = True
    vadFilesFolder: str = ''
    nSensorPerNode: list = field(default_factory=list)
    loadFrom: str = ''
    generateRandomWASNwithSeed: int = 0
    SROperNode: np.ndarray = field(default_factory=lambda: np.array([0]))
    topologyParams: TopologyParameters = field(default_factory=TopologyParameters)
    selfnoiseSNR: float = 50.
    addedNoiseSignalsPerNode: list = field(default_factory=list)
    sensorToNodeIndicesASC: list = field(default_factory=list)
    nSensorPerNodeASC: list = field(default_factory=list)

    def __post_init__(self):
        self.topologyParams.__post_init__()
        self.nNodes = len(self.nSensorPerNode)
        self.nSensorPerNode = np.asarray(self.nSensorPerNode, dtype=int)
        if np.ndim(self.SROperNode) == 0 or len(np.atleast_1d(self.SROperNode)) == 1:
            self.SROperNode = np.full(self.nNodes, float(np.atleast_1d(self.SROperNode)[0]))
        self.SROperNode = np.asarray(self.SROperNode, dtype=float)
        if len(self.SROperNode) != self.nNodes:
            raise ValueError('`SROperNode` must have one entry per node.')
        if len(self.addedNoiseSignalsPerNode) == 0:
            self.addedNoiseSignalsPerNode = np.zeros(self.nNodes, dtype=int)
        self.addedNoiseSignalsPerNode = np.asarray(self.addedNoiseSignalsPerNode, dtype=int)
        self.sensorToNodeIndices = np.array(
            [k for k in range(self.nNodes) for _ in range(int(self.nSensorPerNode[k]))], dtype=int)
        self.VADenergyFactor = 10 ** (self.VADenergyDecrease_dB / 10)


@dataclass
class ExportParameters:
    filterNormsPlot: bool = True
    conditionNumberPlot: bool = True
    convergencePlot: bool = True
    wavFiles: bool = True
    acousticScenarioPlot: bool = True
    sroEstimPerfPlot: bool = True
    metricsPlot: bool = True
    waveformsAndSpectrograms: bool = True
    mmsePerfPlot: bool = False
    mseBatchPerfPlot: bool = False
    bestPerfReference: bool = True
    danseOutputsFile: bool = True
    metricsFile: bool = True
    parametersFile: bool = True
    filterNorms: bool = True
    filters: bool = False
    bypassAllExports: bool = False
    bypassGlobalPickleExport: bool = False
    exportFolder: str = ''
    metricsInPlots: list = field(default_factory=list)
    writeOverPrevious: bool = False

    def __post_init__(self):
        if len(self.metricsInPlots) == 0:
            self.metricsInPlots = ['snr', 'estoi']

    def check_export_folder(self):
        """Exports are out of scope: always run."""
        return True


@dataclass
class TestParameters:
    """``danse_toolbox/d_classes.py:198-324``."""
    __test__ = False   # not a pytest class
    referenceSensor: int = 0
    wasnParams: WASNparameters = field(default_factory=WASNparameters)
    danseParams: DANSEparameters = field(default_factory=DANSEparameters)
    exportParams: ExportParameters = field(default_factory=ExportParameters)
    setThoseSensorsToNoise: list = field(default_factory=list)
    seed: int = 12345
    snrYlimMax: float = None
    loadedFromYaml: bool = False
    originYaml: str = ''

    def __post_init__(self):
        self.wasnParams.__post_init__()
        self.danseParams.__post_init__()
        np.random.seed(self.seed)
        random.seed(self.seed)
        self.testid = self.get_id()
        if self.danseParams.nodeUpdating == 'sim' and any(self.wasnParams.SROperNode != 0):
            raise ValueError('Simultaneous node-updating impossible in the presence of SROs.')
        self.danseParams.saveConditionNumber = bool(self.exportParams.conditionNumberPlot)
        if self.is_fully_connected_wasn() and self.danseParams.compensateSROs and \
                self.danseParams.compensationStrategy == 'network-wide':
            raise ValueError('Network-wide SRO compensation strategy not supported in fully-connected WASNs. Aborting.')
        if not self.is_fully_connected_wasn():
            if 'topo-indep' not in self.danseParams.nodeUpdating:
                self.danseParams.nodeUpdating = f'topo-indep_{self.danseParams.nodeUpdating}'
            self.danseParams.computeSingleSensorBroadcast = False
        var = self.danseParams.startComputeMetricsAt
        if 'after' in var and 'beginning' not in var:
            if 'ms' in var:
                dur = float(var[len('after_'):-2]) / 1e3
            else:
                dur = float(var[len('after_'):-1])
            if dur > self.wasnParams.sigDur:
                raise ValueError('`danseParams.startComputeMetricsAt` is after the end of the signal.')

    def get_id(self):
        return (f'J{self.wasnParams.nNodes}Mk{list(self.wasnParams.nSensorPerNode)}'
                f'WNn{self.wasnParams.nNoiseSources}Nd{self.wasnParams.nDesiredSources}'
                f'T60_{int(self.wasnParams.t60 * 1e3)}ms')

    def is_fully_connected_wasn(self):
        """String comparison only, as the reference (quirk Q1,
        ``d_classes.py:302-303``)."""
        return self.wasnParams.topologyParams.topologyType == 'fully-connected'

    def is_batch(self):
        return self.danseParams.simType == 'batch'

    def load_from_yaml(self, path) -> 'TestParameters':
        self.loadedFromYaml = True
        self.originYaml = path
        out = load_from_yaml(path, self)
        out.__post_init__()
        return out


def load_from_yaml(path, myDataclass):
    """``danse_toolbox/dataclass_methods.py:258-329``: YAML -> nested
    dataclass, ``'[...]'`` strings literal-eval'd, list fields typed
    ``np.ndarray`` converted, then every ``__post_init__`` re-run.  Unlike the
    reference, sub-dataclass instances are per-instance (no shared mutable
    class defaults)."""
    with open(path, 'r') as f:
        d = yaml.load(f, Loader=yaml.SafeLoader)

    def _interpret_lists(d):
        for key in d:
            if type(d[key]) is str and len(d[key]) >= 2 and d[key][0] == '[' and d[key][-1] == ']':
                d[key] = ast.literal_eval(d[key])
            elif type(d[key]) is dict:
                d[key] = _interpret_lists(d[key])
        return d

    d = _interpret_lists(d)

    def _load(d, obj):
        types_ = {f.name: f.type for f in fields(obj)}
        for key, val in d.items():
            if type(val) is dict:
                setattr(obj, key, _load(val, getattr(obj, key)))
            else:
                if type(val) is list and types_.get(key) in (np.ndarray, 'np.ndarray'):
                    val = np.array(val)
                setattr(obj, key, val)
        return obj

    myDataclass = _load(d, myDataclass)
    if hasattr(myDataclass, '__post_init__'):
        myDataclass.__post_init__()
    for k, v in myDataclass.__dict__.items():
        if is_dataclass(v) and hasattr(v, '__post_init__'):
            v.__post_init__()
    return myDataclass
