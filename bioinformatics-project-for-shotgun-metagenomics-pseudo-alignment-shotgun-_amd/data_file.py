"""FASTA / FASTQ files (drop-in for src/data_file.py): extension check, plain or
gzip text, parsed into the containers of records.py -- by the native
multi-threaded parser (libpa.so pa_parse_file) when the file is in its
canonical subset, else by the exact regex grammar of records.py."""

from __future__ import annotations

import gzip
import pickle
from typing import Optional, Set

from records import FASTAQRecordContainer, FASTARecordContainer, NoRecordsInData, RecordContainer


class InvalidExtensionError(Exception):
    def __init__(self, message: str = "") -> None:
        super().__init__(message)


class NoRecordsInDataFile(Exception):
    def __init__(self, message: str = "") -> None:
        super().__init__(message)


class DataFile:
    """Base: subclasses set EXTENSIONS and the container type."""

    EXTENSIONS: Optional[Set[str]] = None

    def __init__(self, file_path: str) -> None:
        self.check_extension(file_path)
        self.container: RecordContainer = self.get_container_type()
        self.parse_file(file_path)

    @classmethod
    def check_extension(cls, file_path: str) -> None:
        if not cls.EXTENSIONS:
            raise NotImplementedError("EXTENSIONS must be defined.")
        if not any(file_path.endswith(ext) for ext in cls.EXTENSIONS):
            raise InvalidExtensionError(f"Invalid file extension. Expected one of {cls.EXTENSIONS}, got {file_path}")

    def get_container_type(self) -> RecordContainer:
        raise NotImplementedError("This method must be implemented in subclasses.")

    NATIVE_KIND: Optional[int] = None  # pa_native.PA_FASTA / PA_FASTQ

    def parse_file(self, file_path: str) -> None:
        # the native parser reads the file itself (mmap / zlib, host threads);
        # None -> outside its canonical subset or unreadable: the exact path below
        if self.NATIVE_KIND is not None and len(self.container) == 0:
            import pa_native
            cols = pa_native.parse_file(self.NATIVE_KIND, file_path)
            if cols is not None:
                self.container.load_columns(cols)
                return
        try:
            self.container.parse_records(self.load_file(file_path))
        except NoRecordsInData:
            raise NoRecordsInDataFile(f"No valid records found in file: {file_path}")

    def load_file(self, file_path: str) -> str:
        opener = gzip.open if file_path.endswith(".gz") else open
        with opener(file_path, "rt", encoding="utf-8") as f:
            return f.read()

    def dump(self, output_file: str) -> None:
        with open(output_file, "wb") as f:
            pickle.dump(self.container, f)


class FASTAFile(DataFile):
    EXTENSIONS = {".fa", ".fa.gz"}
    NATIVE_KIND = 0

    def get_container_type(self) -> FASTARecordContainer:
        return FASTARecordContainer()


class FASTAQFile(DataFile):
    EXTENSIONS = {".fq", ".fq.gz"}
    NATIVE_KIND = 1

    def get_container_type(self) -> FASTAQRecordContainer:
        return FASTAQRecordContainer()
