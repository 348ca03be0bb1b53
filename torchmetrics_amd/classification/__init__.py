"""Classification module metrics (parity: reference ``S/classification/__init__.py``)."""
from torchmetrics_amd.classification.accuracy import Accuracy, BinaryAccuracy, MulticlassAccuracy, MultilabelAccuracy
from torchmetrics_amd.classification.confusion_matrix import (
    BinaryCohenKappa,
    BinaryConfusionMatrix,
    BinaryJaccardIndex,
    BinaryMatthewsCorrCoef,
    CohenKappa,
    ConfusionMatrix,
    JaccardIndex,
    MatthewsCorrCoef,
    MulticlassCohenKappa,
    MulticlassConfusionMatrix,
    MulticlassJaccardIndex,
    MulticlassMatthewsCorrCoef,
    MultilabelConfusionMatrix,
    MultilabelJaccardIndex,
    MultilabelMatthewsCorrCoef,
)
from torchmetrics_amd.classification.extras import (
    BinaryCalibrationError,
    BinaryFairness,
    BinaryGroupStatRates,
    BinaryHingeLoss,
    CalibrationError,
    Dice,
    ExactMatch,
    HingeLoss,
    MulticlassCalibrationError,
    MulticlassExactMatch,
    MulticlassHingeLoss,
    MultilabelCoverageError,
    MultilabelExactMatch,
    MultilabelRankingAveragePrecision,
    MultilabelRankingLoss,
)
from torchmetrics_amd.classification.f_beta import (
    BinaryF1Score,
    BinaryFBetaScore,
    F1Score,
    FBetaScore,
    MulticlassF1Score,
    MulticlassFBetaScore,
    MultilabelF1Score,
    MultilabelFBetaScore,
)
from torchmetrics_amd.classification.fixed_point import (
    BinaryPrecisionAtFixedRecall,
    BinaryRecallAtFixedPrecision,
    BinarySensitivityAtSpecificity,
    BinarySpecificityAtSensitivity,
    MulticlassPrecisionAtFixedRecall,
    MulticlassRecallAtFixedPrecision,
    MulticlassSensitivityAtSpecificity,
    MulticlassSpecificityAtSensitivity,
    MultilabelPrecisionAtFixedRecall,
    MultilabelRecallAtFixedPrecision,
    MultilabelSensitivityAtSpecificity,
    MultilabelSpecificityAtSensitivity,
    PrecisionAtFixedRecall,
    RecallAtFixedPrecision,
    SensitivityAtSpecificity,
    SpecificityAtSensitivity,
)
from torchmetrics_amd.classification.precision_recall_curve import (
    AUROC,
    ROC,
    AveragePrecision,
    BinaryAUROC,
    BinaryAveragePrecision,
    BinaryPrecisionRecallCurve,
    BinaryROC,
    MulticlassAUROC,
    MulticlassAveragePrecision,
    MulticlassPrecisionRecallCurve,
    MulticlassROC,
    MultilabelAUROC,
    MultilabelAveragePrecision,
    MultilabelPrecisionRecallCurve,
    MultilabelROC,
    PrecisionRecallCurve,
)
from torchmetrics_amd.classification.hamming import (
    BinaryHammingDistance,
    HammingDistance,
    MulticlassHammingDistance,
    MultilabelHammingDistance,
)
from torchmetrics_amd.classification.precision_recall import (
    BinaryPrecision,
    BinaryRecall,
    MulticlassPrecision,
    MulticlassRecall,
    MultilabelPrecision,
    MultilabelRecall,
    Precision,
    Recall,
)
from torchmetrics_amd.classification.specificity import (
    BinarySpecificity,
    MulticlassSpecificity,
    MultilabelSpecificity,
    Specificity,
)
from torchmetrics_amd.classification.stat_scores import (
    BinaryStatScores,
    MulticlassStatScores,
    MultilabelStatScores,
    StatScores,
)

__all__ = [k for k in dir() if k[0].isupper()]
