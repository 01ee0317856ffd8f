from .trainer import Trainer, TrainerState, TrainingArguments, TrainOutput, set_seed

__all__ = ["Trainer", "TrainerState", "TrainingArguments", "TrainOutput", "set_seed"]
